#!/usr/bin/env python3
"""Generate dispatch_probe.hip: cycles per threaded-interpreter dispatch on
gfx950 for several glue variants (tools only, not part of the library).

Each kernel runs a wave through NIT x 4 dispatches of 4 handlers that jump to
each other (H0 -> H1 -> H2 -> H3 -> H0): every handler = glue + BODY v_add_f32
on 8 registers. Variants switch glue parts on/off."""
VARIANTS = {
    "rl1_fall": (1, False, "fall"),
    "rl2_fall": (2, False, "fall"),
    "rlconst4_fall": (-4, False, "fall"),
    "smem_fall": ("smem", False, "fall"),
    "smem_lds_fall": ("smem", True, "fall"),
    "salu4_fall": ("salu", False, "fall"),
    # name: (readlanes, lds_prefetch, jump)  jump: 'table' (setpc->s_branch), 'direct' (setpc), 'fall' (no jump)
    "full_table": (4, True, "table"),
    "full_direct": (4, True, "direct"),
    "nolds_table": (4, False, "table"),
    "nolds_direct": (4, False, "direct"),
    "norl_nolds_direct": (0, False, "direct"),
    "fall_body_only": (0, False, "fall"),
    "rl_nolds_fall": (4, False, "fall"),
    "lds_fall": (0, True, "fall"),
}
BODY = 8

def kernel(name, nrl, lds, jump):
    A = []
    a = A.append
    a("s_getpc_b64 s[68:69]")
    a(".Lpc%=:")
    a("s_add_u32 s68, s68, .Ltbl%=-.Lpc%=")
    a("s_addc_u32 s69, s69, 0")
    a("s_mov_b32 s71, s69")
    # v40 = absolute table slot per lane: lane j -> handler (j+1)%4 ; v41 = lane+1 mod 4 ; lane address v42
    a("v_and_b32 v41, 3, v43")          # v43 = lane id input
    a("v_add_u32 v41, 1, v41")
    a("v_and_b32 v41, 3, v41")          # next handler index
    if jump == "table":
        a("v_lshlrev_b32 v40, 2, v41")
    else:
        # direct: absolute handler addresses from a small table of offsets
        a("v_lshlrev_b32 v40, 2, v41")   # placeholder; fixed below via s_branch targets not known -> use table
    a("v_add_u32 v40, s68, v40")
    a("v_mov_b32 v44, v41")             # pn: next index (cyclic)
    a("s_mov_b32 s66, 0")
    a("s_mov_b32 s84, 0")
    a("s_mov_b32 s80, %[it]")              # iterations
    a("s_nop 4")
    a("v_readlane_b32 s70, v40, 3")     # handler 0 slot (lane 3 -> index 0)
    a("s_nop 4")
    if jump == "fall":
        a("s_branch .Lh0%=")
    else:
        a("s_setpc_b64 s[70:71]")
    a(".Ltbl%=:")
    for k in range(4):
        a(f"s_branch .Lh{k}%=")
    for k in range(4):
        a(f".Lh{k}%=:")
        if nrl == "smem":
            a("s_waitcnt lgkmcnt(0)")
            a("s_load_dwordx4 s[76:79], s[82:83], s84")
            a("s_add_u32 s84, s84, 16")
            a("s_and_b32 s84, s84, 255")
        elif nrl == "salu":
            a("s_add_u32 s73, s73, 3")
            a("s_add_u32 s65, s65, 5")
            a("s_add_u32 s66, s66, 1")
            a("s_and_b32 s66, s66, 63")
        elif nrl < 0:
            for q in range(-nrl):
                a(f"v_readlane_b32 s{[73,70,65,77][q]}, v42, {q + 5}")
        else:
            if nrl >= 1: a("v_readlane_b32 s73, v42, s66")
            if nrl >= 2: a("v_readlane_b32 s70, v40, s66")
            if nrl >= 3: a("v_readlane_b32 s65, v42, s66")
            if nrl >= 4: a("v_readlane_b32 s66, v44, s66")
        if lds:
            a("v_add_u32 v0, s73, v42" if (nrl and nrl not in ("smem", "salu")) else "v_add_u32 v0, 0, v42")
            dst = 48 if k % 2 == 0 else 56
            a(f"ds_read_b128 v[{dst}:{dst+3}], v0")
            a(f"ds_read_b128 v[{dst+4}:{dst+7}], v0 offset:1024")
            a("s_waitcnt lgkmcnt(2)")
        src = 56 if k % 2 == 0 else 48
        for r in range(BODY):
            a(f"v_add_f32 v{32+r}, v{32+r}, v{src + r}")
        if k == 3:
            a("s_sub_u32 s80, s80, 1")
            a("s_cbranch_scc1 .Ldone%=")
        if jump == "fall":
            if k == 3:
                a("s_branch .Lh0%=")
        elif jump == "table":
            if nrl < 2:
                a(f"s_add_u32 s70, s68, {4*((k+1)%4)}")
            a("s_setpc_b64 s[70:71]")
        else:  # direct
            a(f"s_branch .Lh{(k+1)%4}%=")  # emulate a direct jump with a plain branch
    a(".Ldone%=:")
    a("s_waitcnt lgkmcnt(0)")
    text = "\\n".join(A)
    clob = ",".join(f'"v{r}"' for r in [0] + list(range(40, 42)) + [44] + list(range(48, 64))) + \
           ',"s65","s66","s68","s69","s70","s71","s73","s76","s77","s78","s79","s80","s84","scc"'
    return f'''
__global__ void __launch_bounds__(256) {name}(float* out, int iters) {{
  extern __shared__ float sm[];
  for (int i = threadIdx.x; i < 4096; i += 256) sm[i] = i * 0.5f;
  __syncthreads();
  float acc0 = threadIdx.x, acc1 = 1, acc2 = 2, acc3 = 3, acc4 = 4, acc5 = 5, acc6 = 6, acc7 = 7;
  unsigned lane = threadIdx.x & 63, la = (threadIdx.x & 63) * 16;
  asm volatile("{text}" : "+{{v32}}"(acc0), "+{{v33}}"(acc1), "+{{v34}}"(acc2), "+{{v35}}"(acc3), "+{{v36}}"(acc4), "+{{v37}}"(acc5), "+{{v38}}"(acc6), "+{{v39}}"(acc7)
     : "{{v43}}"(lane), [it] "s"(iters), "{{v42}}"(la), "{{s[82:83]}}"(out) : {clob});
  float s = acc0 + acc1 + acc2 + acc3 + acc4 + acc5 + acc6 + acc7;
  if (s == 1234.5f) out[threadIdx.x] = s;
}}
'''

src = ['#include <hip/hip_runtime.h>', '#include <cstdio>', '#include <cstdlib>',
       '#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s line %d\\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)']
for n, (nrl, lds, jump) in VARIANTS.items():
    src.append(kernel(n, nrl, lds, jump))
src.append('''
template <typename K>
void run(const char* name, K k, float* d, int occ) {
  const int iters = 2000;
  hipEvent_t a, b; CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  dim3 grid(256 * occ), block(256);
  hipLaunchKernelGGL(k, grid, block, 16384, 0, d, 4);
  CHECK(hipEventRecord(a));
  hipLaunchKernelGGL(k, grid, block, 16384, 0, d, iters);
  CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b));
  float ms; CHECK(hipEventElapsedTime(&ms, a, b));
  const double cyc = ms * 1e-3 * 2.4e9 / (iters * 4.0);
  printf("%-20s occ=%d  %8.1f cyc/dispatch/SIMD  (%7.1f per wave-dispatch)\\n", name, occ, cyc, cyc / occ);
}
int main() {
  float* d; CHECK(hipMalloc(&d, 4096));
  for (int occ : {1, 2, 4, 8}) {''')
for n in VARIANTS:
    src.append(f'    run("{n}", {n}, d, occ);')
src.append('''  }
  CHECK(hipFree(d));
  return 0;
}''')
open("dispatch_probe.hip", "w").write("\n".join(src) + "\n")
