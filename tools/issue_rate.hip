// issue_rate.hip — VALU issue cost on gfx950 (tools/, not part of the library).
//
// Settles how many SIMD cycles one wave64 VALU instruction occupies when
// 1, 2, 4 or 8 waves share a SIMD (VERDICT r02 "What's weak" 3): the tree
// code's 4-cycle vs 2-cycle accounting decides whether cutting VALU
// instructions or hiding latency / fetch is the lever.
//
// Each kernel runs a loop whose body is 64 instructions of one kind over 8
// independent register chains (ILP 8) or 1 chain (dependent, latency view).
// Occupancy is pinned with dynamic LDS: a workgroup of 256 threads (one wave
// per SIMD) asks for 160 KiB / W, so at most W workgroups share a CU; the
// grid is 256 CUs x W workgroups. Reported per config:
//   cyc/inst/SIMD (chip) = kernel_time * f_clk * 1024 SIMDs / wave-instructions
//   cyc/inst (wave)      = s_memtime delta of one wave / its instructions
// f_clk is measured in-kernel from s_memtime (shader clock) against
// s_memrealtime (100 MHz).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                           \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__);          \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

enum Op { ADD, FMA, PK_ADD, PK_FMA, PK_MUL, EXP, RCP, FMA64, LSHLADD, MAX3, CNDMASK, MIX_PK_EXP, NOP,
          MOV, MUL, MAXF, CMP, XOR, ADDU, CVT64, RNDNE, LDEXP, PKMOV, MED3, CND2, LSHL, BFI, CVTI, MULF64, ADD_ABS,
          MIX_F32_EXP, MIX_PK_MAX3, MAX_ABS, FMAC, CMP64 };
static const char* kName[] = {"v_add_f32", "v_fma_f32", "v_pk_add_f32", "v_pk_fma_f32", "v_pk_mul_f32",
                              "v_exp_f32", "v_rcp_f32", "v_fma_f64", "v_lshl_add_u32", "v_max3_f32",
                              "v_cndmask_b32", "4 v_pk_fma_f32 + 1 v_exp_f32 (ILP1: pk_fma)", "s_nop 0",
                              "v_mov_b32", "v_mul_f32 (VOP2)", "v_max_f32 (VOP2)", "v_cmp_lt_f32 (VOPC)",
                              "v_xor_b32", "v_add_u32", "v_cvt_f32_f64", "v_rndne_f32", "v_ldexp_f32",
                              "v_pk_mov_b32", "v_med3_f32", "v_cndmask_b32 (VOP2)", "v_lshlrev_b32", "v_bfi_b32",
                              "v_cvt_i32_f32", "v_mul_f64", "v_add_f32 |a|+|b| (VOP3)",
                              "4 v_fma_f32 + 1 v_exp_f32", "2 v_pk_fma_f32 + 1 v_max3_f32",
                              "v_max_f32 |a|,|b| (VOP3)", "v_fmac_f32 (VOP2)", "v_cmp_gt_f32 |a| -> sgpr (VOP3)"};

// The loop body: 64 instructions of one kind in ONE asm statement (no
// compiler-inserted s_nop between them), over 8 independent chains (ILP 8:
// instruction j works on chain j % 8) or 1 chain (ILP 1).
#define R8(x) x x x x x x x x
#define B8(a0, a1, a2, a3, a4, a5, a6, a7) a0 a1 a2 a3 a4 a5 a6 a7
template <int OP, int ILP>
__device__ __forceinline__ void body(float (&v)[8], double (&pv)[8], double (&d)[8]) {
#define V8(ins) asm volatile(R8(B8(ins("%0"), ins("%1"), ins("%2"), ins("%3"), ins("%4"), ins("%5"), ins("%6"), ins("%7"))) \
                              : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]))
#define P8(ins, arr) asm volatile(R8(B8(ins("%0"), ins("%1"), ins("%2"), ins("%3"), ins("%4"), ins("%5"), ins("%6"), ins("%7"))) \
                              : "+v"(arr[0]), "+v"(arr[1]), "+v"(arr[2]), "+v"(arr[3]), "+v"(arr[4]), "+v"(arr[5]), "+v"(arr[6]), "+v"(arr[7]))
#define V1(ins) asm volatile(R8(R8(ins("%0"))) : "+v"(v[0]))
#define P1(ins, arr) asm volatile(R8(R8(ins("%0"))) : "+v"(arr[0]))
#define I_ADD(r) "v_add_f32 " r ", 1.0, " r "\n"
#define I_FMA(r) "v_fma_f32 " r ", " r ", 0.5, 1.0\n"
#define I_PKADD(r) "v_pk_add_f32 " r ", " r ", " r "\n"
#define I_PKFMA(r) "v_pk_fma_f32 " r ", " r ", " r ", " r "\n"
#define I_PKMUL(r) "v_pk_mul_f32 " r ", " r ", " r "\n"
#define I_EXP(r) "v_exp_f32 " r ", " r "\n"
#define I_RCP(r) "v_rcp_f32 " r ", " r "\n"
#define I_FMA64(r) "v_fma_f64 " r ", " r ", 0.5, 1.0\n"
#define I_LSHLADD(r) "v_lshl_add_u32 " r ", " r ", 3, " r "\n"
#define I_MAX3(r) "v_max3_f32 " r ", " r ", |" r "|, 1.0\n"
#define I_CND(r) "v_cndmask_b32 " r ", " r ", 1.0, vcc\n"
#define I_NOP(r) "s_nop 0\n"
#define I_MIX(r) "v_pk_fma_f32 " r ", " r ", " r ", " r "\n"
#define I_MOV(r) "v_mov_b32 " r ", " r "\n"
#define I_MUL(r) "v_mul_f32 " r ", " r ", " r "\n"
#define I_MAXF(r) "v_max_f32 " r ", " r ", " r "\n"
#define I_CMP(r) "v_cmp_lt_f32 vcc, " r ", " r "\n"
#define I_XOR(r) "v_xor_b32 " r ", " r ", " r "\n"
#define I_ADDU(r) "v_add_u32 " r ", " r ", " r "\n"
#define I_RNDNE(r) "v_rndne_f32 " r ", " r "\n"
#define I_LDEXP(r) "v_ldexp_f32 " r ", " r ", 3\n"
#define I_MED3(r) "v_med3_f32 " r ", " r ", " r ", 1.0\n"
#define I_CND2(r) "v_cndmask_b32 " r ", " r ", " r ", vcc\n"
#define I_LSHL(r) "v_lshlrev_b32 " r ", 1, " r "\n"
#define I_BFI(r) "v_bfi_b32 " r ", " r ", " r ", " r "\n"
#define I_CVTI(r) "v_cvt_i32_f32 " r ", " r "\n"
#define I_ADDABS(r) "v_add_f32_e64 " r ", |" r "|, |" r "|\n"
#define I_MULF64(r) "v_mul_f64 " r ", " r ", " r "\n"
#define I_MAXABS(r) "v_max_f32_e64 " r ", |" r "|, |" r "|\n"
#define I_FMAC(r) "v_fmac_f32 " r ", " r ", " r "\n"
#define I_CMP64(r) "v_cmp_gt_f32_e64 s[2:3], |" r "|, " r "\n"
#define I_PKMOV(r) "v_pk_mov_b32 " r ", " r ", " r " op_sel:[0,1]\n"
  if constexpr (ILP == 8) {
    if constexpr (OP == ADD) V8(I_ADD);
    else if constexpr (OP == FMA) V8(I_FMA);
    else if constexpr (OP == PK_ADD) P8(I_PKADD, pv);
    else if constexpr (OP == PK_FMA) P8(I_PKFMA, pv);
    else if constexpr (OP == PK_MUL) P8(I_PKMUL, pv);
    else if constexpr (OP == EXP) V8(I_EXP);
    else if constexpr (OP == RCP) V8(I_RCP);
    else if constexpr (OP == FMA64) P8(I_FMA64, d);
    else if constexpr (OP == LSHLADD) V8(I_LSHLADD);
    else if constexpr (OP == MAX3) V8(I_MAX3);
    else if constexpr (OP == CNDMASK) V8(I_CND);
    else if constexpr (OP == MIX_PK_EXP) {  // 4 packed fmas then 1 exp, independent chains
      asm volatile(R8("v_pk_fma_f32 %0, %0, %0, %0\n v_pk_fma_f32 %1, %1, %1, %1\n v_pk_fma_f32 %2, %2, %2, %2\n"
                      " v_pk_fma_f32 %3, %3, %3, %3\n v_exp_f32 %4, %4\n")
                   : "+v"(pv[0]), "+v"(pv[1]), "+v"(pv[2]), "+v"(pv[3]), "+v"(v[0]));
    } else if constexpr (OP == MOV) V8(I_MOV);
    else if constexpr (OP == MUL) V8(I_MUL);
    else if constexpr (OP == MAXF) V8(I_MAXF);
    else if constexpr (OP == CMP) V8(I_CMP);
    else if constexpr (OP == XOR) V8(I_XOR);
    else if constexpr (OP == ADDU) V8(I_ADDU);
    else if constexpr (OP == CVT64) {  // f32 <- f64: 8 independent pairs
      asm volatile(R8("v_cvt_f32_f64 %0, %8\n v_cvt_f32_f64 %1, %9\n v_cvt_f32_f64 %2, %10\n v_cvt_f32_f64 %3, %11\n"
                      " v_cvt_f32_f64 %4, %12\n v_cvt_f32_f64 %5, %13\n v_cvt_f32_f64 %6, %14\n v_cvt_f32_f64 %7, %15\n")
                   : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7])
                   : "v"(d[0]), "v"(d[1]), "v"(d[2]), "v"(d[3]), "v"(d[4]), "v"(d[5]), "v"(d[6]), "v"(d[7]));
    } else if constexpr (OP == RNDNE) V8(I_RNDNE);
    else if constexpr (OP == LDEXP) V8(I_LDEXP);
    else if constexpr (OP == PKMOV) P8(I_PKMOV, pv);
    else if constexpr (OP == MED3) V8(I_MED3);
    else if constexpr (OP == CND2) V8(I_CND2);
    else if constexpr (OP == LSHL) V8(I_LSHL);
    else if constexpr (OP == BFI) V8(I_BFI);
    else if constexpr (OP == CVTI) V8(I_CVTI);
    else if constexpr (OP == MULF64) P8(I_MULF64, d);
    else if constexpr (OP == ADD_ABS) V8(I_ADDABS);
    else if constexpr (OP == MAX_ABS) V8(I_MAXABS);
    else if constexpr (OP == FMAC) V8(I_FMAC);
    else if constexpr (OP == CMP64) { asm volatile(R8(B8(I_CMP64("%0"), I_CMP64("%1"), I_CMP64("%2"), I_CMP64("%3"), I_CMP64("%4"), I_CMP64("%5"), I_CMP64("%6"), I_CMP64("%7"))) :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7]) : "s2", "s3"); }
    else if constexpr (OP == MIX_F32_EXP) {  // 4 scalar fmas then 1 exp
      asm volatile(R8("v_fma_f32 %0, %0, %0, %0\n v_fma_f32 %1, %1, %1, %1\n v_fma_f32 %2, %2, %2, %2\n"
                      " v_fma_f32 %3, %3, %3, %3\n v_exp_f32 %4, %4\n")
                   : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]));
    } else if constexpr (OP == MIX_PK_MAX3) {  // 2 packed fmas then 1 max3
      asm volatile(R8("v_pk_fma_f32 %0, %0, %0, %0\n v_pk_fma_f32 %1, %1, %1, %1\n v_max3_f32 %2, %2, |%2|, 1.0\n")
                   : "+v"(pv[0]), "+v"(pv[1]), "+v"(v[0]));
    } else V8(I_NOP);
  } else {
    if constexpr (OP == ADD) V1(I_ADD);
    else if constexpr (OP == FMA) V1(I_FMA);
    else if constexpr (OP == PK_ADD) P1(I_PKADD, pv);
    else if constexpr (OP == PK_FMA) P1(I_PKFMA, pv);
    else if constexpr (OP == PK_MUL) P1(I_PKMUL, pv);
    else if constexpr (OP == EXP) V1(I_EXP);
    else if constexpr (OP == RCP) V1(I_RCP);
    else if constexpr (OP == FMA64) P1(I_FMA64, d);
    else if constexpr (OP == LSHLADD) V1(I_LSHLADD);
    else if constexpr (OP == MAX3) V1(I_MAX3);
    else if constexpr (OP == CNDMASK) V1(I_CND);
    else if constexpr (OP == MIX_PK_EXP) P1(I_MIX, pv);
    else V1(I_NOP);
  }
}

template <int OP, int ILP>
__global__ void __launch_bounds__(256) probe(unsigned long long* cyc, unsigned long long* rt, float* sink, int iters) {
  extern __shared__ float lds[];
  float v[8];
  double d[8], pv[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    v[i] = threadIdx.x * 1e-3f + i * 0.25f;
    pv[i] = threadIdx.x * 1e-3 + i * 0.5;
    d[i] = threadIdx.x * 1e-3 + i;
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) body<OP, ILP>(v, pv, d);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) acc += v[i] + (float)d[i] + (float)pv[i];
  if (threadIdx.x % 64 == 0) {
    const int w = blockIdx.x * 4 + threadIdx.x / 64;
    cyc[w] = t1 - t0;
    rt[w] = r1 - r0;
  }
  if (acc == 1234.5f) { lds[threadIdx.x] = acc; sink[threadIdx.x] = lds[(threadIdx.x + 1) % 256]; }
}

typedef void (*KFn)(unsigned long long*, unsigned long long*, float*, int);

template <int OP>
static KFn pick(int ilp) { return ilp == 1 ? probe<OP, 1> : probe<OP, 8>; }

static KFn kernel_for(int op, int ilp) {
  switch (op) {
    case ADD: return pick<ADD>(ilp);
    case FMA: return pick<FMA>(ilp);
    case PK_ADD: return pick<PK_ADD>(ilp);
    case PK_FMA: return pick<PK_FMA>(ilp);
    case PK_MUL: return pick<PK_MUL>(ilp);
    case EXP: return pick<EXP>(ilp);
    case RCP: return pick<RCP>(ilp);
    case FMA64: return pick<FMA64>(ilp);
    case LSHLADD: return pick<LSHLADD>(ilp);
    case MAX3: return pick<MAX3>(ilp);
    case CNDMASK: return pick<CNDMASK>(ilp);
    case MIX_PK_EXP: return pick<MIX_PK_EXP>(ilp);
    case MOV: return pick<MOV>(ilp);
    case MUL: return pick<MUL>(ilp);
    case MAXF: return pick<MAXF>(ilp);
    case CMP: return pick<CMP>(ilp);
    case XOR: return pick<XOR>(ilp);
    case ADDU: return pick<ADDU>(ilp);
    case CVT64: return pick<CVT64>(ilp);
    case RNDNE: return pick<RNDNE>(ilp);
    case LDEXP: return pick<LDEXP>(ilp);
    case PKMOV: return pick<PKMOV>(ilp);
    case MED3: return pick<MED3>(ilp);
    case CND2: return pick<CND2>(ilp);
    case LSHL: return pick<LSHL>(ilp);
    case BFI: return pick<BFI>(ilp);
    case CVTI: return pick<CVTI>(ilp);
    case MULF64: return pick<MULF64>(ilp);
    case ADD_ABS: return pick<ADD_ABS>(ilp);
    case MIX_F32_EXP: return pick<MIX_F32_EXP>(ilp);
    case MIX_PK_MAX3: return pick<MIX_PK_MAX3>(ilp);
    case MAX_ABS: return pick<MAX_ABS>(ilp);
    case FMAC: return pick<FMAC>(ilp);
    case CMP64: return pick<CMP64>(ilp);
    default: return pick<NOP>(ilp);
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  const int nsimd = ncu * 4;
  const int maxw = 8;
  unsigned long long *d_cyc, *d_rt;
  float* d_sink;
  CHECK(hipMalloc(&d_cyc, sizeof(unsigned long long) * ncu * maxw * 4));
  CHECK(hipMalloc(&d_rt, sizeof(unsigned long long) * ncu * maxw * 4));
  CHECK(hipMalloc(&d_sink, 256 * sizeof(float)));
  unsigned long long* h_cyc = new unsigned long long[ncu * maxw * 4];
  unsigned long long* h_rt = new unsigned long long[ncu * maxw * 4];
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::printf("# %d CUs; iters %d x 64 instructions per wave; one 256-thread workgroup = one wave per SIMD\n", ncu,
              iters);
  std::printf("%-30s %4s %3s %10s %10s %12s %12s\n", "instruction", "ilp", "W", "kernel_ms", "f_clk_GHz",
              "cyc/inst/SIMD", "cyc/inst(wave)");
  // argv[2] == "ext": the second table (ILP 8 only)
  const bool ext = argc > 2 && std::strcmp(argv[2], "ext") == 0;
  std::vector<int> ops = {NOP, ADD, FMA, PK_ADD, PK_FMA, PK_MUL, EXP, RCP, FMA64, LSHLADD, MAX3, CNDMASK, MIX_PK_EXP};
  if (ext) ops = {MOV, MUL, MAXF, CMP, XOR, ADDU, CVT64, RNDNE, LDEXP, PKMOV, MED3, CND2, LSHL, BFI, CVTI, MULF64,
                  ADD_ABS, MIX_F32_EXP, MIX_PK_MAX3, MAX_ABS, FMAC, CMP64};
  const int ws[] = {1, 2, 4, 5, 8};
  for (int op : ops) {
    for (int ilp : {8, 1}) {
      if (ext && ilp == 1) continue;
      for (int W : ws) {
        KFn k = kernel_for(op, ilp);
        const size_t lds = (size_t)(160 * 1024 / W) / 256 * 256 - 256;
        CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024));
        const int grid = ncu * W;
        hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, 0, d_cyc, d_rt, d_sink, 10);  // warm
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, 0, d_cyc, d_rt, d_sink, iters);
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms = 0.f;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const int nw = grid * 4;
        CHECK(hipMemcpy(h_cyc, d_cyc, sizeof(unsigned long long) * nw, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(h_rt, d_rt, sizeof(unsigned long long) * nw, hipMemcpyDeviceToHost));
        double sc = 0, sr = 0, cmax = 0;
        for (int i = 0; i < nw; ++i) {
          sc += (double)h_cyc[i];
          sr += (double)h_rt[i];
          if ((double)h_cyc[i] > cmax) cmax = (double)h_cyc[i];
        }
        const double f = sr > 0 ? sc / sr * 100e6 : 0;  // shader cycles per 100 MHz tick
        // instructions per loop iteration: 64, except the mixes (5 x 8 and 3 x 8)
        const int per_it = (ilp == 8 && (op == MIX_PK_EXP || op == MIX_F32_EXP)) ? 40
                           : (ilp == 8 && op == MIX_PK_MAX3) ? 24 : 64;
        const double inst_per_wave = (double)iters * per_it;
        const double wave_inst = inst_per_wave * nw;
        const double chip = (double)ms * 1e-3 * f * nsimd / wave_inst;
        const double wave = sc / nw / inst_per_wave;
        std::printf("%-30s %4d %3d %10.3f %10.3f %12.2f %12.2f\n", kName[op], ilp, W, ms, f / 1e9, chip, wave);
        std::fflush(stdout);
      }
    }
  }
  return 0;
}
