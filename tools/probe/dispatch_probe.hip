#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

__global__ void __launch_bounds__(256) rl1_fall(float* out, int iters) {
  extern __shared__ float sm[];
  for (int i = threadIdx.x; i < 4096; i += 256) sm[i] = i * 0.5f;
  __syncthreads();
  float acc0 = threadIdx.x, acc1 = 1, acc2 = 2, acc3 = 3, acc4 = 4, acc5 = 5, acc6 = 6, acc7 = 7;
  unsigned lane = threadIdx.x & 63, la = (threadIdx.x & 63) * 16;
  asm volatile("s_getpc_b64 s[68:69]\n.Lpc%=:\ns_add_u32 s68, s68, .Ltbl%=-.Lpc%=\ns_addc_u32 s69, s69, 0\ns_mov_b32 s71, s69\nv_and_b32 v41, 3, v43\nv_add_u32 v41, 1, v41\nv_and_b32 v41, 3, v41\nv_lshlrev_b32 v40, 2, v41\nv_add_u32 v40, s68, v40\nv_mov_b32 v44, v41\ns_mov_b32 s66, 0\ns_mov_b32 s84, 0\ns_mov_b32 s80, %[it]\ns_nop 4\nv_readlane_b32 s70, v40, 3\ns_nop 4\ns_branch .Lh0%=\n.Ltbl%=:\ns_branch .Lh0%=\ns_branch .Lh1%=\ns_branch .Lh2%=\ns_branch .Lh3%=\n.Lh0%=:\nv_readlane_b32 s73, v42, s66\nv_add_f32 v32, v32, v56\nv_add_f32 v33, v33, v57\nv_add_f32 v34, v34, v58\nv_add_f32 v35, v35, v59\nv_add_f32 v36, v36, v60\nv_add_f32 v37, v37, v61\nv_add_f32 v38, v38, v62\nv_add_f32 v39, v39, v63\n.Lh1%=:\nv_readlane_b32 s73, v42, s66\nv_add_f32 v32, v32, v48\nv_add_f32 v33, v33, v49\nv_add_f32 v34, v34, v50\nv_add_f32 v35, v35, v51\nv_add_f32 v36, v36, v52\nv_add_f32 v37, v37, v53\nv_add_f32 v38, v38, v54\nv_add_f32 v39, v39, v55\n.Lh2%=:\nv_readlane_b32 s73, v42, s66\nv_add_f32 v32, v32, v56\nv_add_f32 v33, v33, v57\nv_add_f32 v34, v34, v58\nv_add_f32 v35, v35, v59\nv_add_f32 v36, v36, v60\nv_add_f32 v37, v37, v61\nv_add_f32 v38, v38, v62\nv_add_f32 v39, v39, v63\n.Lh3%=:\nv_readlane_b32 s73, v42, s66\nv_add_f32 v32, v32, v48\nv_add_f32 v33, v33, v49\nv_add_f32 v34, v34, v50\nv_add_f32 v35, v35, v51\nv_add_f32 v36, v36, v52\nv_add_f32 v37, v37, v53\nv_add_f32 v38, v38, v54\nv_add_f32 v39, v39, v55\ns_sub_u32 s80, s80, 1\ns_cbranch_scc1 .Ldone%=\ns_branch .Lh0%=\n.Ldone%=:\ns_waitcnt lgkmcnt(0)" : "+{v32}"(acc0), "+{v33}"(acc1), "+{v34}"(acc2), "+{v35}"(acc3), "+{v36}"(acc4), "+{v37}"(acc5), "+{v38}"(acc6), "+{v39}"(acc7)
     : "{v43}"(lane), [it] "s"(iters), "{v42}"(la), "{s[82:83]}"(out) : "v0","v40","v41","v44","v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63","s65","s66","s68","s69","s70","s71","s73","s76","s77","s78","s79","s80","s84","scc");
  float s = acc0 + acc1 + acc2 + acc3 + acc4 + acc5 + acc6 + acc7;
  if (s == 1234.5f) out[threadIdx.x] = s;
}


__global__ void __launch_bounds__(256) rl2_fall(float* out, int iters) {
  extern __shared__ float sm[];
  for (int i = threadIdx.x; i < 4096; i += 256) sm[i] = i * 0.5f;
  __syncthreads();
  float acc0 = threadIdx.x, acc1 = 1, acc2 = 2, acc3 = 3, acc4 = 4, acc5 = 5, acc6 = 6, acc7 = 7;
  unsigned lane = threadIdx.x & 63, la = (threadIdx.x & 63) * 16;
  asm volatile("s_getpc_b64 s[68:69]\n.Lpc%=:\ns_add_u32 s68, s68, .Ltbl%=-.Lpc%=\ns_addc_u32 s69, s69, 0\ns_mov_b32 s71, s69\nv_and_b32 v41, 3, v43\nv_add_u32 v41, 1, v41\nv_and_b32 v41, 3, v41\nv_lshlrev_b32 v40, 2, v41\nv_add_u32 v40, s68, v40\nv_mov_b32 v44, v41\ns_mov_b32 s66, 0\ns_mov_b32 s84, 0\ns_mov_b32 s80, %[it]\ns_nop 4\nv_readlane_b32 s70, v40, 3\ns_nop 4\ns_branch .Lh0%=\n.Ltbl%=:\ns_branch .Lh0%=\ns_branch .Lh1%=\ns_branch .Lh2%=\ns_branch .Lh3%=\n.Lh0%=:\nv_readlane_b32 s73, v42, s66\nv_readlane_b32 s70, v40, s66\nv_add_f32 v32, v32, v56\nv_add_f32 v33, v33, v57\nv_add_f32 v34, v34, v58\nv_add_f32 v35, v35, v59\nv_add_f32 v36, v36, v60\nv_add_f32 v37, v37, v61\nv_add_f32 v38, v38, v62\nv_add_f32 v39, v39, v63\n.Lh1%=:\nv_readlane_b32 s73, v42, s66\nv_readlane_b32 s70, v40, s66\nv_add_f32 v32, v32, v48\nv_add_f32 v33, v33, v49\nv_add_f32 v34, v34, v50\nv_add_f32 v35, v35, v51\nv_add_f32 v36, v36, v52\nv_add_f32 v37, v37, v53\nv_add_f32 v38, v38, v54\nv_add_f32 v39, v39, v55\n.Lh2%=:\nv_readlane_b32 s73, v42, s66\nv_readlane_b32 s70, v40, s66\nv_add_f32 v32, v32, v56\nv_add_f32 v33, v33, v57\nv_add_f32 v34, v34, v58\nv_add_f32 v35, v35, v59\nv_add_f32 v36, v36, v60\nv_add_f32 v37, v37, v61\nv_add_f32 v38, v38, v62\nv_add_f32 v39, v39, v63\n.Lh3%=:\nv_readlane_b32 s73, v42, s66\nv_readlane_b32 s70, v40, s66\nv_add_f32 v32, v32, v48\nv_add_f32 v33, v33, v49\nv_add_f32 v34, v34, v50\nv_add_f32 v35, v35, v51\nv_add_f32 v36, v36, v52\nv_add_f32 v37, v37, v53\nv_add_f32 v38, v38, v54\nv_add_f32 v39, v39, v55\ns_sub_u32 s80, s80, 1\ns_cbranch_scc1 .Ldone%=\ns_branch .Lh0%=\n.Ldone%=:\ns_waitcnt lgkmcnt(0)" : "+{v32}"(acc0), "+{v33}"(acc1), "+{v34}"(acc2), "+{v35}"(acc3), "+{v36}"(acc4), "+{v37}"(acc5), "+{v38}"(acc6), "+{v39}"(acc7)
     : "{v43}"(lane), [it] "s"(iters), "{v42}"(la), "{s[82:83]}"(out) : "v0","v40","v41","v44","v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63","s65","s66","s68","s69","s70","s71","s73","s76","s77","s78","s79","s80","s84","scc");
  float s = acc0 + acc1 + acc2 + acc3 + acc4 + acc5 + acc6 + acc7;
  if (s == 1234.5f) out[threadIdx.x] = s;
}


__global__ void __launch_bounds__(256) rlconst4_fall(float* out, int iters) {
  extern __shared__ float sm[];
  for (int i = threadIdx.x; i < 4096; i += 256) sm[i] = i * 0.5f;
  __syncthreads();
  float acc0 = threadIdx.x, acc1 = 1, acc2 = 2, acc3 = 3, acc4 = 4, acc5 = 5, acc6 = 6, acc7 = 7;
  unsigned lane = threadIdx.x & 63, la = (threadIdx.x & 63) * 16;
  asm volatile("s_getpc_b64 s[68:69]\n.Lpc%=:\ns_add_u32 s68, s68, .Ltbl%=-.Lpc%=\ns_addc_u32 s69, s69, 0\ns_mov_b32 s71, s69\nv_and_b32 v41, 3, v43\nv_add_u32 v41, 1, v41\nv_and_b32 v41, 3, v41\nv_lshlrev_b32 v40, 2, v41\nv_add_u32 v40, s68, v40\nv_mov_b32 v44, v41\ns_mov_b32 s66, 0\ns_mov_b32 s84, 0\ns_mov_b32 s80, %[it]\ns_nop 4\nv_readlane_b32 s70, v40, 3\ns_nop 4\ns_branch .Lh0%=\n.Ltbl%=:\ns_branch .Lh0%=\ns_branch .Lh1%=\ns_branch .Lh2%=\ns_branch .Lh3%=\n.Lh0%=:\nv_readlane_b32 s73, v42, 5\nv_readlane_b32 s70, v42, 6\nv_readlane_b32 s65, v42, 7\nv_readlane_b32 s77, v42, 8\nv_add_f32 v32, v32, v56\nv_add_f32 v33, v33, v57\nv_add_f32 v34, v34, v58\nv_add_f32 v35, v35, v59\nv_add_f32 v36, v36, v60\nv_add_f32 v37, v37, v61\nv_add_f32 v38, v38, v62\nv_add_f32 v39, v39, v63\n.Lh1%=:\nv_readlane_b32 s73, v42, 5\nv_readlane_b32 s70, v42, 6\nv_readlane_b32 s65, v42, 7\nv_readlane_b32 s77, v42, 8\nv_add_f32 v32, v32, v48\nv_add_f32 v33, v33, v49\nv_add_f32 v34, v34, v50\nv_add_f32 v35, v35, v51\nv_add_f32 v36, v36, v52\nv_add_f32 v37, v37, v53\nv_add_f32 v38, v38, v54\nv_add_f32 v39, v39, v55\n.Lh2%=:\nv_readlane_b32 s73, v42, 5\nv_readlane_b32 s70, v42, 6\nv_readlane_b32 s65, v42, 7\nv_readlane_b32 s77, v42, 8\nv_add_f32 v32, v32, v56\nv_add_f32 v33, v33, v57\nv_add_f32 v34, v34, v58\nv_add_f32 v35, v35, v59\nv_add_f32 v36, v36, v60\nv_add_f32 v37, v37, v61\nv_add_f32 v38, v38, v62\nv_add_f32 v39, v39, v63\n.Lh3%=:\nv_readlane_b32 s73, v42, 5\nv_readlane_b32 s70, v42, 6\nv_readlane_b32 s65, v42, 7\nv_readlane_b32 s77, v42, 8\nv_add_f32 v32, v32, v48\nv_add_f32 v33, v33, v49\nv_add_f32 v34, v34, v50\nv_add_f32 v35, v35, v51\nv_add_f32 v36, v36, v52\nv_add_f32 v37, v37, v53\nv_add_f32 v38, v38, v54\nv_add_f32 v39, v39, v55\ns_sub_u32 s80, s80, 1\ns_cbranch_scc1 .Ldone%=\ns_branch .Lh0%=\n.Ldone%=:\ns_waitcnt lgkmcnt(0)" : "+{v32}"(acc0), "+{v33}"(acc1), "+{v34}"(acc2), "+{v35}"(acc3), "+{v36}"(acc4), "+{v37}"(acc5), "+{v38}"(acc6), "+{v39}"(acc7)
     : "{v43}"(lane), [it] "s"(iters), "{v42}"(la), "{s[82:83]}"(out) : "v0","v40","v41","v44","v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63","s65","s66","s68","s69","s70","s71","s73","s76","s77","s78","s79","s80","s84","scc");
  float s = acc0 + acc1 + acc2 + acc3 + acc4 + acc5 + acc6 + acc7;
  if (s == 1234.5f) out[threadIdx.x] = s;
}


__global__ void __launch_bounds__(256) smem_fall(float* out, int iters) {
  extern __shared__ float sm[];
  for (int i = threadIdx.x; i < 4096; i += 256) sm[i] = i * 0.5f;
  __syncthreads();
  float acc0 = threadIdx.x, acc1 = 1, acc2 = 2, acc3 = 3, acc4 = 4, acc5 = 5, acc6 = 6, acc7 = 7;
  unsigned lane = threadIdx.x & 63, la = (threadIdx.x & 63) * 16;
  asm volatile("s_getpc_b64 s[68:69]\n.Lpc%=:\ns_add_u32 s68, s68, .Ltbl%=-.Lpc%=\ns_addc_u32 s69, s69, 0\ns_mov_b32 s71, s69\nv_and_b32 v41, 3, v43\nv_add_u32 v41, 1, v41\nv_and_b32 v41, 3, v41\nv_lshlrev_b32 v40, 2, v41\nv_add_u32 v40, s68, v40\nv_mov_b32 v44, v41\ns_mov_b32 s66, 0\ns_mov_b32 s84, 0\ns_mov_b32 s80, %[it]\ns_nop 4\nv_readlane_b32 s70, v40, 3\ns_nop 4\ns_branch .Lh0%=\n.Ltbl%=:\ns_branch .Lh0%=\ns_branch .Lh1%=\ns_branch .Lh2%=\ns_branch .Lh3%=\n.Lh0%=:\ns_waitcnt lgkmcnt(0)\ns_load_dwordx4 s[76:79], s[82:83], s84\ns_add_u32 s84, s84, 16\ns_and_b32 s84, s84, 255\nv_add_f32 v32, v32, v56\nv_add_f32 v33, v33, v57\nv_add_f32 v34, v34, v58\nv_add_f32 v35, v35, v59\nv_add_f32 v36, v36, v60\nv_add_f32 v37, v37, v61\nv_add_f32 v38, v38, v62\nv_add_f32 v39, v39, v63\n.Lh1%=:\ns_waitcnt lgkmcnt(0)\ns_load_dwordx4 s[76:79], s[82:83], s84\ns_add_u32 s84, s84, 16\ns_and_b32 s84, s84, 255\nv_add_f32 v32, v32, v48\nv_add_f32 v33, v33, v49\nv_add_f32 v34, v34, v50\nv_add_f32 v35, v35, v51\nv_add_f32 v36, v36, v52\nv_add_f32 v37, v37, v53\nv_add_f32 v38, v38, v54\nv_add_f32 v39, v39, v55\n.Lh2%=:\ns_waitcnt lgkmcnt(0)\ns_load_dwordx4 s[76:79], s[82:83], s84\ns_add_u32 s84, s84, 16\ns_and_b32 s84, s84, 255\nv_add_f32 v32, v32, v56\nv_add_f32 v33, v33, v57\nv_add_f32 v34, v34, v58\nv_add_f32 v35, v35, v59\nv_add_f32 v36, v36, v60\nv_add_f32 v37, v37, v61\nv_add_f32 v38, v38, v62\nv_add_f32 v39, v39, v63\n.Lh3%=:\ns_waitcnt lgkmcnt(0)\ns_load_dwordx4 s[76:79], s[82:83], s84\ns_add_u32 s84, s84, 16\ns_and_b32 s84, s84, 255\nv_add_f32 v32, v32, v48\nv_add_f32 v33, v33, v49\nv_add_f32 v34, v34, v50\nv_add_f32 v35, v35, v51\nv_add_f32 v36, v36, v52\nv_add_f32 v37, v37, v53\nv_add_f32 v38, v38, v54\nv_add_f32 v39, v39, v55\ns_sub_u32 s80, s80, 1\ns_cbranch_scc1 .Ldone%=\ns_branch .Lh0%=\n.Ldone%=:\ns_waitcnt lgkmcnt(0)" : "+{v32}"(acc0), "+{v33}"(acc1), "+{v34}"(acc2), "+{v35}"(acc3), "+{v36}"(acc4), "+{v37}"(acc5), "+{v38}"(acc6), "+{v39}"(acc7)
     : "{v43}"(lane), [it] "s"(iters), "{v42}"(la), "{s[82:83]}"(out) : "v0","v40","v41","v44","v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63","s65","s66","s68","s69","s70","s71","s73","s76","s77","s78","s79","s80","s84","scc");
  float s = acc0 + acc1 + acc2 + acc3 + acc4 + acc5 + acc6 + acc7;
  if (s == 1234.5f) out[threadIdx.x] = s;
}


__global__ void __launch_bounds__(256) smem_lds_fall(float* out, int iters) {
  extern __shared__ float sm[];
  for (int i = threadIdx.x; i < 4096; i += 256) sm[i] = i * 0.5f;
  __syncthreads();
  float acc0 = threadIdx.x, acc1 = 1, acc2 = 2, acc3 = 3, acc4 = 4, acc5 = 5, acc6 = 6, acc7 = 7;
  unsigned lane = threadIdx.x & 63, la = (threadIdx.x & 63) * 16;
  asm volatile("s_getpc_b64 s[68:69]\n.Lpc%=:\ns_add_u32 s68, s68, .Ltbl%=-.Lpc%=\ns_addc_u32 s69, s69, 0\ns_mov_b32 s71, s69\nv_and_b32 v41, 3, v43\nv_add_u32 v41, 1, v41\nv_and_b32 v41, 3, v41\nv_lshlrev_b32 v40, 2, v41\nv_add_u32 v40, s68, v40\nv_mov_b32 v44, v41\ns_mov_b32 s66, 0\ns_mov_b32 s84, 0\ns_mov_b32 s80, %[it]\ns_nop 4\nv_readlane_b32 s70, v40, 3\ns_nop 4\ns_branch .Lh0%=\n.Ltbl%=:\ns_branch .Lh0%=\ns_branch .Lh1%=\ns_branch .Lh2%=\ns_branch .Lh3%=\n.Lh0%=:\ns_waitcnt lgkmcnt(0)\ns_load_dwordx4 s[76:79], s[82:83], s84\ns_add_u32 s84, s84, 16\ns_and_b32 s84, s84, 255\nv_add_u32 v0, 0, v42\nds_read_b128 v[48:51], v0\nds_read_b128 v[52:55], v0 offset:1024\ns_waitcnt lgkmcnt(2)\nv_add_f32 v32, v32, v56\nv_add_f32 v33, v33, v57\nv_add_f32 v34, v34, v58\nv_add_f32 v35, v35, v59\nv_add_f32 v36, v36, v60\nv_add_f32 v37, v37, v61\nv_add_f32 v38, v38, v62\nv_add_f32 v39, v39, v63\n.Lh1%=:\ns_waitcnt lgkmcnt(0)\ns_load_dwordx4 s[76:79], s[82:83], s84\ns_add_u32 s84, s84, 16\ns_and_b32 s84, s84, 255\nv_add_u32 v0, 0, v42\nds_read_b128 v[56:59], v0\nds_read_b128 v[60:63], v0 offset:1024\ns_waitcnt lgkmcnt(2)\nv_add_f32 v32, v32, v48\nv_add_f32 v33, v33, v49\nv_add_f32 v34, v34, v50\nv_add_f32 v35, v35, v51\nv_add_f32 v36, v36, v52\nv_add_f32 v37, v37, v53\nv_add_f32 v38, v38, v54\nv_add_f32 v39, v39, v55\n.Lh2%=:\ns_waitcnt lgkmcnt(0)\ns_load_dwordx4 s[76:79], s[82:83], s84\ns_add_u32 s84, s84, 16\ns_and_b32 s84, s84, 255\nv_add_u32 v0, 0, v42\nds_read_b128 v[48:51], v0\nds_read_b128 v[52:55], v0 offset:1024\ns_waitcnt lgkmcnt(2)\nv_add_f32 v32, v32, v56\nv_add_f32 v33, v33, v57\nv_add_f32 v34, v34, v58\nv_add_f32 v35, v35, v59\nv_add_f32 v36, v36, v60\nv_add_f32 v37, v37, v61\nv_add_f32 v38, v38, v62\nv_add_f32 v39, v39, v63\n.Lh3%=:\ns_waitcnt lgkmcnt(0)\ns_load_dwordx4 s[76:79], s[82:83], s84\ns_add_u32 s84, s84, 16\ns_and_b32 s84, s84, 255\nv_add_u32 v0, 0, v42\nds_read_b128 v[56:59], v0\nds_read_b128 v[60:63], v0 offset:1024\ns_waitcnt lgkmcnt(2)\nv_add_f32 v32, v32, v48\nv_add_f32 v33, v33, v49\nv_add_f32 v34, v34, v50\nv_add_f32 v35, v35, v51\nv_add_f32 v36, v36, v52\nv_add_f32 v37, v37, v53\nv_add_f32 v38, v38, v54\nv_add_f32 v39, v39, v55\ns_sub_u32 s80, s80, 1\ns_cbranch_scc1 .Ldone%=\ns_branch .Lh0%=\n.Ldone%=:\ns_waitcnt lgkmcnt(0)" : "+{v32}"(acc0), "+{v33}"(acc1), "+{v34}"(acc2), "+{v35}"(acc3), "+{v36}"(acc4), "+{v37}"(acc5), "+{v38}"(acc6), "+{v39}"(acc7)
     : "{v43}"(lane), [it] "s"(iters), "{v42}"(la), "{s[82:83]}"(out) : "v0","v40","v41","v44","v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63","s65","s66","s68","s69","s70","s71","s73","s76","s77","s78","s79","s80","s84","scc");
  float s = acc0 + acc1 + acc2 + acc3 + acc4 + acc5 + acc6 + acc7;
  if (s == 1234.5f) out[threadIdx.x] = s;
}


__global__ void __launch_bounds__(256) salu4_fall(float* out, int iters) {
  extern __shared__ float sm[];
  for (int i = threadIdx.x; i < 4096; i += 256) sm[i] = i * 0.5f;
  __syncthreads();
  float acc0 = threadIdx.x, acc1 = 1, acc2 = 2, acc3 = 3, acc4 = 4, acc5 = 5, acc6 = 6, acc7 = 7;
  unsigned lane = threadIdx.x & 63, la = (threadIdx.x & 63) * 16;
  asm volatile("s_getpc_b64 s[68:69]\n.Lpc%=:\ns_add_u32 s68, s68, .Ltbl%=-.Lpc%=\ns_addc_u32 s69, s69, 0\ns_mov_b32 s71, s69\nv_and_b32 v41, 3, v43\nv_add_u32 v41, 1, v41\nv_and_b32 v41, 3, v41\nv_lshlrev_b32 v40, 2, v41\nv_add_u32 v40, s68, v40\nv_mov_b32 v44, v41\ns_mov_b32 s66, 0\ns_mov_b32 s84, 0\ns_mov_b32 s80, %[it]\ns_nop 4\nv_readlane_b32 s70, v40, 3\ns_nop 4\ns_branch .Lh0%=\n.Ltbl%=:\ns_branch .Lh0%=\ns_branch .Lh1%=\ns_branch .Lh2%=\ns_branch .Lh3%=\n.Lh0%=:\ns_add_u32 s73, s73, 3\ns_add_u32 s65, s65, 5\ns_add_u32 s66, s66, 1\ns_and_b32 s66, s66, 63\nv_add_f32 v32, v32, v56\nv_add_f32 v33, v33, v57\nv_add_f32 v34, v34, v58\nv_add_f32 v35, v35, v59\nv_add_f32 v36, v36, v60\nv_add_f32 v37, v37, v61\nv_add_f32 v38, v38, v62\nv_add_f32 v39, v39, v63\n.Lh1%=:\ns_add_u32 s73, s73, 3\ns_add_u32 s65, s65, 5\ns_add_u32 s66, s66, 1\ns_and_b32 s66, s66, 63\nv_add_f32 v32, v32, v48\nv_add_f32 v33, v33, v49\nv_add_f32 v34, v34, v50\nv_add_f32 v35, v35, v51\nv_add_f32 v36, v36, v52\nv_add_f32 v37, v37, v53\nv_add_f32 v38, v38, v54\nv_add_f32 v39, v39, v55\n.Lh2%=:\ns_add_u32 s73, s73, 3\ns_add_u32 s65, s65, 5\ns_add_u32 s66, s66, 1\ns_and_b32 s66, s66, 63\nv_add_f32 v32, v32, v56\nv_add_f32 v33, v33, v57\nv_add_f32 v34, v34, v58\nv_add_f32 v35, v35, v59\nv_add_f32 v36, v36, v60\nv_add_f32 v37, v37, v61\nv_add_f32 v38, v38, v62\nv_add_f32 v39, v39, v63\n.Lh3%=:\ns_add_u32 s73, s73, 3\ns_add_u32 s65, s65, 5\ns_add_u32 s66, s66, 1\ns_and_b32 s66, s66, 63\nv_add_f32 v32, v32, v48\nv_add_f32 v33, v33, v49\nv_add_f32 v34, v34, v50\nv_add_f32 v35, v35, v51\nv_add_f32 v36, v36, v52\nv_add_f32 v37, v37, v53\nv_add_f32 v38, v38, v54\nv_add_f32 v39, v39, v55\ns_sub_u32 s80, s80, 1\ns_cbranch_scc1 .Ldone%=\ns_branch .Lh0%=\n.Ldone%=:\ns_waitcnt lgkmcnt(0)" : "+{v32}"(acc0), "+{v33}"(acc1), "+{v34}"(acc2), "+{v35}"(acc3), "+{v36}"(acc4), "+{v37}"(acc5), "+{v38}"(acc6), "+{v39}"(acc7)
     : "{v43}"(lane), [it] "s"(iters), "{v42}"(la), "{s[82:83]}"(out) : "v0","v40","v41","v44","v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63","s65","s66","s68","s69","s70","s71","s73","s76","s77","s78","s79","s80","s84","scc");
  float s = acc0 + acc1 + acc2 + acc3 + acc4 + acc5 + acc6 + acc7;
  if (s == 1234.5f) out[threadIdx.x] = s;
}


__global__ void __launch_bounds__(256) full_table(float* out, int iters) {
  extern __shared__ float sm[];
  for (int i = threadIdx.x; i < 4096; i += 256) sm[i] = i * 0.5f;
  __syncthreads();
  float acc0 = threadIdx.x, acc1 = 1, acc2 = 2, acc3 = 3, acc4 = 4, acc5 = 5, acc6 = 6, acc7 = 7;
  unsigned lane = threadIdx.x & 63, la = (threadIdx.x & 63) * 16;
  asm volatile("s_getpc_b64 s[68:69]\n.Lpc%=:\ns_add_u32 s68, s68, .Ltbl%=-.Lpc%=\ns_addc_u32 s69, s69, 0\ns_mov_b32 s71, s69\nv_and_b32 v41, 3, v43\nv_add_u32 v41, 1, v41\nv_and_b32 v41, 3, v41\nv_lshlrev_b32 v40, 2, v41\nv_add_u32 v40, s68, v40\nv_mov_b32 v44, v41\ns_mov_b32 s66, 0\ns_mov_b32 s84, 0\ns_mov_b32 s80, %[it]\ns_nop 4\nv_readlane_b32 s70, v40, 3\ns_nop 4\ns_setpc_b64 s[70:71]\n.Ltbl%=:\ns_branch .Lh0%=\ns_branch .Lh1%=\ns_branch .Lh2%=\ns_branch .Lh3%=\n.Lh0%=:\nv_readlane_b32 s73, v42, s66\nv_readlane_b32 s70, v40, s66\nv_readlane_b32 s65, v42, s66\nv_readlane_b32 s66, v44, s66\nv_add_u32 v0, s73, v42\nds_read_b128 v[48:51], v0\nds_read_b128 v[52:55], v0 offset:1024\ns_waitcnt lgkmcnt(2)\nv_add_f32 v32, v32, v56\nv_add_f32 v33, v33, v57\nv_add_f32 v34, v34, v58\nv_add_f32 v35, v35, v59\nv_add_f32 v36, v36, v60\nv_add_f32 v37, v37, v61\nv_add_f32 v38, v38, v62\nv_add_f32 v39, v39, v63\ns_setpc_b64 s[70:71]\n.Lh1%=:\nv_readlane_b32 s73, v42, s66\nv_readlane_b32 s70, v40, s66\nv_readlane_b32 s65, v42, s66\nv_readlane_b32 s66, v44, s66\nv_add_u32 v0, s73, v42\nds_read_b128 v[56:59], v0\nds_read_b128 v[60:63], v0 offset:1024\ns_waitcnt lgkmcnt(2)\nv_add_f32 v32, v32, v48\nv_add_f32 v33, v33, v49\nv_add_f32 v34, v34, v50\nv_add_f32 v35, v35, v51\nv_add_f32 v36, v36, v52\nv_add_f32 v37, v37, v53\nv_add_f32 v38, v38, v54\nv_add_f32 v39, v39, v55\ns_setpc_b64 s[70:71]\n.Lh2%=:\nv_readlane_b32 s73, v42, s66\nv_readlane_b32 s70, v40, s66\nv_readlane_b32 s65, v42, s66\nv_readlane_b32 s66, v44, s66\nv_add_u32 v0, s73, v42\nds_read_b128 v[48:51], v0\nds_read_b128 v[52:55], v0 offset:1024\ns_waitcnt lgkmcnt(2)\nv_add_f32 v32, v32, v56\nv_add_f32 v33, v33, v57\nv_add_f32 v34, v34, v58\nv_add_f32 v35, v35, v59\nv_add_f32 v36, v36, v60\nv_add_f32 v37, v37, v61\nv_add_f32 v38, v38, v62\nv_add_f32 v39, v39, v63\ns_setpc_b64 s[70:71]\n.Lh3%=:\nv_readlane_b32 s73, v42, s66\nv_readlane_b32 s70, v40, s66\nv_readlane_b32 s65, v42, s66\nv_readlane_b32 s66, v44, s66\nv_add_u32 v0, s73, v42\nds_read_b128 v[56:59], v0\nds_read_b128 v[60:63], v0 offset:1024\ns_waitcnt lgkmcnt(2)\nv_add_f32 v32, v32, v48\nv_add_f32 v33, v33, v49\nv_add_f32 v34, v34, v50\nv_add_f32 v35, v35, v51\nv_add_f32 v36, v36, v52\nv_add_f32 v37, v37, v53\nv_add_f32 v38, v38, v54\nv_add_f32 v39, v39, v55\ns_sub_u32 s80, s80, 1\ns_cbranch_scc1 .Ldone%=\ns_setpc_b64 s[70:71]\n.Ldone%=:\ns_waitcnt lgkmcnt(0)" : "+{v32}"(acc0), "+{v33}"(acc1), "+{v34}"(acc2), "+{v35}"(acc3), "+{v36}"(acc4), "+{v37}"(acc5), "+{v38}"(acc6), "+{v39}"(acc7)
     : "{v43}"(lane), [it] "s"(iters), "{v42}"(la), "{s[82:83]}"(out) : "v0","v40","v41","v44","v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63","s65","s66","s68","s69","s70","s71","s73","s76","s77","s78","s79","s80","s84","scc");
  float s = acc0 + acc1 + acc2 + acc3 + acc4 + acc5 + acc6 + acc7;
  if (s == 1234.5f) out[threadIdx.x] = s;
}


__global__ void __launch_bounds__(256) full_direct(float* out, int iters) {
  extern __shared__ float sm[];
  for (int i = threadIdx.x; i < 4096; i += 256) sm[i] = i * 0.5f;
  __syncthreads();
  float acc0 = threadIdx.x, acc1 = 1, acc2 = 2, acc3 = 3, acc4 = 4, acc5 = 5, acc6 = 6, acc7 = 7;
  unsigned lane = threadIdx.x & 63, la = (threadIdx.x & 63) * 16;
  asm volatile("s_getpc_b64 s[68:69]\n.Lpc%=:\ns_add_u32 s68, s68, .Ltbl%=-.Lpc%=\ns_addc_u32 s69, s69, 0\ns_mov_b32 s71, s69\nv_and_b32 v41, 3, v43\nv_add_u32 v41, 1, v41\nv_and_b32 v41, 3, v41\nv_lshlrev_b32 v40, 2, v41\nv_add_u32 v40, s68, v40\nv_mov_b32 v44, v41\ns_mov_b32 s66, 0\ns_mov_b32 s84, 0\ns_mov_b32 s80, %[it]\ns_nop 4\nv_readlane_b32 s70, v40, 3\ns_nop 4\ns_setpc_b64 s[70:71]\n.Ltbl%=:\ns_branch .Lh0%=\ns_branch .Lh1%=\ns_branch .Lh2%=\ns_branch .Lh3%=\n.Lh0%=:\nv_readlane_b32 s73, v42, s66\nv_readlane_b32 s70, v40, s66\nv_readlane_b32 s65, v42, s66\nv_readlane_b32 s66, v44, s66\nv_add_u32 v0, s73, v42\nds_read_b128 v[48:51], v0\nds_read_b128 v[52:55], v0 offset:1024\ns_waitcnt lgkmcnt(2)\nv_add_f32 v32, v32, v56\nv_add_f32 v33, v33, v57\nv_add_f32 v34, v34, v58\nv_add_f32 v35, v35, v59\nv_add_f32 v36, v36, v60\nv_add_f32 v37, v37, v61\nv_add_f32 v38, v38, v62\nv_add_f32 v39, v39, v63\ns_branch .Lh1%=\n.Lh1%=:\nv_readlane_b32 s73, v42, s66\nv_readlane_b32 s70, v40, s66\nv_readlane_b32 s65, v42, s66\nv_readlane_b32 s66, v44, s66\nv_add_u32 v0, s73, v42\nds_read_b128 v[56:59], v0\nds_read_b128 v[60:63], v0 offset:1024\ns_waitcnt lgkmcnt(2)\nv_add_f32 v32, v32, v48\nv_add_f32 v33, v33, v49\nv_add_f32 v34, v34, v50\nv_add_f32 v35, v35, v51\nv_add_f32 v36, v36, v52\nv_add_f32 v37, v37, v53\nv_add_f32 v38, v38, v54\nv_add_f32 v39, v39, v55\ns_branch .Lh2%=\n.Lh2%=:\nv_readlane_b32 s73, v42, s66\nv_readlane_b32 s70, v40, s66\nv_readlane_b32 s65, v42, s66\nv_readlane_b32 s66, v44, s66\nv_add_u32 v0, s73, v42\nds_read_b128 v[48:51], v0\nds_read_b128 v[52:55], v0 offset:1024\ns_waitcnt lgkmcnt(2)\nv_add_f32 v32, v32, v56\nv_add_f32 v33, v33, v57\nv_add_f32 v34, v34, v58\nv_add_f32 v35, v35, v59\nv_add_f32 v36, v36, v60\nv_add_f32 v37, v37, v61\nv_add_f32 v38, v38, v62\nv_add_f32 v39, v39, v63\ns_branch .Lh3%=\n.Lh3%=:\nv_readlane_b32 s73, v42, s66\nv_readlane_b32 s70, v40, s66\nv_readlane_b32 s65, v42, s66\nv_readlane_b32 s66, v44, s66\nv_add_u32 v0, s73, v42\nds_read_b128 v[56:59], v0\nds_read_b128 v[60:63], v0 offset:1024\ns_waitcnt lgkmcnt(2)\nv_add_f32 v32, v32, v48\nv_add_f32 v33, v33, v49\nv_add_f32 v34, v34, v50\nv_add_f32 v35, v35, v51\nv_add_f32 v36, v36, v52\nv_add_f32 v37, v37, v53\nv_add_f32 v38, v38, v54\nv_add_f32 v39, v39, v55\ns_sub_u32 s80, s80, 1\ns_cbranch_scc1 .Ldone%=\ns_branch .Lh0%=\n.Ldone%=:\ns_waitcnt lgkmcnt(0)" : "+{v32}"(acc0), "+{v33}"(acc1), "+{v34}"(acc2), "+{v35}"(acc3), "+{v36}"(acc4), "+{v37}"(acc5), "+{v38}"(acc6), "+{v39}"(acc7)
     : "{v43}"(lane), [it] "s"(iters), "{v42}"(la), "{s[82:83]}"(out) : "v0","v40","v41","v44","v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63","s65","s66","s68","s69","s70","s71","s73","s76","s77","s78","s79","s80","s84","scc");
  float s = acc0 + acc1 + acc2 + acc3 + acc4 + acc5 + acc6 + acc7;
  if (s == 1234.5f) out[threadIdx.x] = s;
}


__global__ void __launch_bounds__(256) nolds_table(float* out, int iters) {
  extern __shared__ float sm[];
  for (int i = threadIdx.x; i < 4096; i += 256) sm[i] = i * 0.5f;
  __syncthreads();
  float acc0 = threadIdx.x, acc1 = 1, acc2 = 2, acc3 = 3, acc4 = 4, acc5 = 5, acc6 = 6, acc7 = 7;
  unsigned lane = threadIdx.x & 63, la = (threadIdx.x & 63) * 16;
  asm volatile("s_getpc_b64 s[68:69]\n.Lpc%=:\ns_add_u32 s68, s68, .Ltbl%=-.Lpc%=\ns_addc_u32 s69, s69, 0\ns_mov_b32 s71, s69\nv_and_b32 v41, 3, v43\nv_add_u32 v41, 1, v41\nv_and_b32 v41, 3, v41\nv_lshlrev_b32 v40, 2, v41\nv_add_u32 v40, s68, v40\nv_mov_b32 v44, v41\ns_mov_b32 s66, 0\ns_mov_b32 s84, 0\ns_mov_b32 s80, %[it]\ns_nop 4\nv_readlane_b32 s70, v40, 3\ns_nop 4\ns_setpc_b64 s[70:71]\n.Ltbl%=:\ns_branch .Lh0%=\ns_branch .Lh1%=\ns_branch .Lh2%=\ns_branch .Lh3%=\n.Lh0%=:\nv_readlane_b32 s73, v42, s66\nv_readlane_b32 s70, v40, s66\nv_readlane_b32 s65, v42, s66\nv_readlane_b32 s66, v44, s66\nv_add_f32 v32, v32, v56\nv_add_f32 v33, v33, v57\nv_add_f32 v34, v34, v58\nv_add_f32 v35, v35, v59\nv_add_f32 v36, v36, v60\nv_add_f32 v37, v37, v61\nv_add_f32 v38, v38, v62\nv_add_f32 v39, v39, v63\ns_setpc_b64 s[70:71]\n.Lh1%=:\nv_readlane_b32 s73, v42, s66\nv_readlane_b32 s70, v40, s66\nv_readlane_b32 s65, v42, s66\nv_readlane_b32 s66, v44, s66\nv_add_f32 v32, v32, v48\nv_add_f32 v33, v33, v49\nv_add_f32 v34, v34, v50\nv_add_f32 v35, v35, v51\nv_add_f32 v36, v36, v52\nv_add_f32 v37, v37, v53\nv_add_f32 v38, v38, v54\nv_add_f32 v39, v39, v55\ns_setpc_b64 s[70:71]\n.Lh2%=:\nv_readlane_b32 s73, v42, s66\nv_readlane_b32 s70, v40, s66\nv_readlane_b32 s65, v42, s66\nv_readlane_b32 s66, v44, s66\nv_add_f32 v32, v32, v56\nv_add_f32 v33, v33, v57\nv_add_f32 v34, v34, v58\nv_add_f32 v35, v35, v59\nv_add_f32 v36, v36, v60\nv_add_f32 v37, v37, v61\nv_add_f32 v38, v38, v62\nv_add_f32 v39, v39, v63\ns_setpc_b64 s[70:71]\n.Lh3%=:\nv_readlane_b32 s73, v42, s66\nv_readlane_b32 s70, v40, s66\nv_readlane_b32 s65, v42, s66\nv_readlane_b32 s66, v44, s66\nv_add_f32 v32, v32, v48\nv_add_f32 v33, v33, v49\nv_add_f32 v34, v34, v50\nv_add_f32 v35, v35, v51\nv_add_f32 v36, v36, v52\nv_add_f32 v37, v37, v53\nv_add_f32 v38, v38, v54\nv_add_f32 v39, v39, v55\ns_sub_u32 s80, s80, 1\ns_cbranch_scc1 .Ldone%=\ns_setpc_b64 s[70:71]\n.Ldone%=:\ns_waitcnt lgkmcnt(0)" : "+{v32}"(acc0), "+{v33}"(acc1), "+{v34}"(acc2), "+{v35}"(acc3), "+{v36}"(acc4), "+{v37}"(acc5), "+{v38}"(acc6), "+{v39}"(acc7)
     : "{v43}"(lane), [it] "s"(iters), "{v42}"(la), "{s[82:83]}"(out) : "v0","v40","v41","v44","v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63","s65","s66","s68","s69","s70","s71","s73","s76","s77","s78","s79","s80","s84","scc");
  float s = acc0 + acc1 + acc2 + acc3 + acc4 + acc5 + acc6 + acc7;
  if (s == 1234.5f) out[threadIdx.x] = s;
}


__global__ void __launch_bounds__(256) nolds_direct(float* out, int iters) {
  extern __shared__ float sm[];
  for (int i = threadIdx.x; i < 4096; i += 256) sm[i] = i * 0.5f;
  __syncthreads();
  float acc0 = threadIdx.x, acc1 = 1, acc2 = 2, acc3 = 3, acc4 = 4, acc5 = 5, acc6 = 6, acc7 = 7;
  unsigned lane = threadIdx.x & 63, la = (threadIdx.x & 63) * 16;
  asm volatile("s_getpc_b64 s[68:69]\n.Lpc%=:\ns_add_u32 s68, s68, .Ltbl%=-.Lpc%=\ns_addc_u32 s69, s69, 0\ns_mov_b32 s71, s69\nv_and_b32 v41, 3, v43\nv_add_u32 v41, 1, v41\nv_and_b32 v41, 3, v41\nv_lshlrev_b32 v40, 2, v41\nv_add_u32 v40, s68, v40\nv_mov_b32 v44, v41\ns_mov_b32 s66, 0\ns_mov_b32 s84, 0\ns_mov_b32 s80, %[it]\ns_nop 4\nv_readlane_b32 s70, v40, 3\ns_nop 4\ns_setpc_b64 s[70:71]\n.Ltbl%=:\ns_branch .Lh0%=\ns_branch .Lh1%=\ns_branch .Lh2%=\ns_branch .Lh3%=\n.Lh0%=:\nv_readlane_b32 s73, v42, s66\nv_readlane_b32 s70, v40, s66\nv_readlane_b32 s65, v42, s66\nv_readlane_b32 s66, v44, s66\nv_add_f32 v32, v32, v56\nv_add_f32 v33, v33, v57\nv_add_f32 v34, v34, v58\nv_add_f32 v35, v35, v59\nv_add_f32 v36, v36, v60\nv_add_f32 v37, v37, v61\nv_add_f32 v38, v38, v62\nv_add_f32 v39, v39, v63\ns_branch .Lh1%=\n.Lh1%=:\nv_readlane_b32 s73, v42, s66\nv_readlane_b32 s70, v40, s66\nv_readlane_b32 s65, v42, s66\nv_readlane_b32 s66, v44, s66\nv_add_f32 v32, v32, v48\nv_add_f32 v33, v33, v49\nv_add_f32 v34, v34, v50\nv_add_f32 v35, v35, v51\nv_add_f32 v36, v36, v52\nv_add_f32 v37, v37, v53\nv_add_f32 v38, v38, v54\nv_add_f32 v39, v39, v55\ns_branch .Lh2%=\n.Lh2%=:\nv_readlane_b32 s73, v42, s66\nv_readlane_b32 s70, v40, s66\nv_readlane_b32 s65, v42, s66\nv_readlane_b32 s66, v44, s66\nv_add_f32 v32, v32, v56\nv_add_f32 v33, v33, v57\nv_add_f32 v34, v34, v58\nv_add_f32 v35, v35, v59\nv_add_f32 v36, v36, v60\nv_add_f32 v37, v37, v61\nv_add_f32 v38, v38, v62\nv_add_f32 v39, v39, v63\ns_branch .Lh3%=\n.Lh3%=:\nv_readlane_b32 s73, v42, s66\nv_readlane_b32 s70, v40, s66\nv_readlane_b32 s65, v42, s66\nv_readlane_b32 s66, v44, s66\nv_add_f32 v32, v32, v48\nv_add_f32 v33, v33, v49\nv_add_f32 v34, v34, v50\nv_add_f32 v35, v35, v51\nv_add_f32 v36, v36, v52\nv_add_f32 v37, v37, v53\nv_add_f32 v38, v38, v54\nv_add_f32 v39, v39, v55\ns_sub_u32 s80, s80, 1\ns_cbranch_scc1 .Ldone%=\ns_branch .Lh0%=\n.Ldone%=:\ns_waitcnt lgkmcnt(0)" : "+{v32}"(acc0), "+{v33}"(acc1), "+{v34}"(acc2), "+{v35}"(acc3), "+{v36}"(acc4), "+{v37}"(acc5), "+{v38}"(acc6), "+{v39}"(acc7)
     : "{v43}"(lane), [it] "s"(iters), "{v42}"(la), "{s[82:83]}"(out) : "v0","v40","v41","v44","v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63","s65","s66","s68","s69","s70","s71","s73","s76","s77","s78","s79","s80","s84","scc");
  float s = acc0 + acc1 + acc2 + acc3 + acc4 + acc5 + acc6 + acc7;
  if (s == 1234.5f) out[threadIdx.x] = s;
}


__global__ void __launch_bounds__(256) norl_nolds_direct(float* out, int iters) {
  extern __shared__ float sm[];
  for (int i = threadIdx.x; i < 4096; i += 256) sm[i] = i * 0.5f;
  __syncthreads();
  float acc0 = threadIdx.x, acc1 = 1, acc2 = 2, acc3 = 3, acc4 = 4, acc5 = 5, acc6 = 6, acc7 = 7;
  unsigned lane = threadIdx.x & 63, la = (threadIdx.x & 63) * 16;
  asm volatile("s_getpc_b64 s[68:69]\n.Lpc%=:\ns_add_u32 s68, s68, .Ltbl%=-.Lpc%=\ns_addc_u32 s69, s69, 0\ns_mov_b32 s71, s69\nv_and_b32 v41, 3, v43\nv_add_u32 v41, 1, v41\nv_and_b32 v41, 3, v41\nv_lshlrev_b32 v40, 2, v41\nv_add_u32 v40, s68, v40\nv_mov_b32 v44, v41\ns_mov_b32 s66, 0\ns_mov_b32 s84, 0\ns_mov_b32 s80, %[it]\ns_nop 4\nv_readlane_b32 s70, v40, 3\ns_nop 4\ns_setpc_b64 s[70:71]\n.Ltbl%=:\ns_branch .Lh0%=\ns_branch .Lh1%=\ns_branch .Lh2%=\ns_branch .Lh3%=\n.Lh0%=:\nv_add_f32 v32, v32, v56\nv_add_f32 v33, v33, v57\nv_add_f32 v34, v34, v58\nv_add_f32 v35, v35, v59\nv_add_f32 v36, v36, v60\nv_add_f32 v37, v37, v61\nv_add_f32 v38, v38, v62\nv_add_f32 v39, v39, v63\ns_branch .Lh1%=\n.Lh1%=:\nv_add_f32 v32, v32, v48\nv_add_f32 v33, v33, v49\nv_add_f32 v34, v34, v50\nv_add_f32 v35, v35, v51\nv_add_f32 v36, v36, v52\nv_add_f32 v37, v37, v53\nv_add_f32 v38, v38, v54\nv_add_f32 v39, v39, v55\ns_branch .Lh2%=\n.Lh2%=:\nv_add_f32 v32, v32, v56\nv_add_f32 v33, v33, v57\nv_add_f32 v34, v34, v58\nv_add_f32 v35, v35, v59\nv_add_f32 v36, v36, v60\nv_add_f32 v37, v37, v61\nv_add_f32 v38, v38, v62\nv_add_f32 v39, v39, v63\ns_branch .Lh3%=\n.Lh3%=:\nv_add_f32 v32, v32, v48\nv_add_f32 v33, v33, v49\nv_add_f32 v34, v34, v50\nv_add_f32 v35, v35, v51\nv_add_f32 v36, v36, v52\nv_add_f32 v37, v37, v53\nv_add_f32 v38, v38, v54\nv_add_f32 v39, v39, v55\ns_sub_u32 s80, s80, 1\ns_cbranch_scc1 .Ldone%=\ns_branch .Lh0%=\n.Ldone%=:\ns_waitcnt lgkmcnt(0)" : "+{v32}"(acc0), "+{v33}"(acc1), "+{v34}"(acc2), "+{v35}"(acc3), "+{v36}"(acc4), "+{v37}"(acc5), "+{v38}"(acc6), "+{v39}"(acc7)
     : "{v43}"(lane), [it] "s"(iters), "{v42}"(la), "{s[82:83]}"(out) : "v0","v40","v41","v44","v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63","s65","s66","s68","s69","s70","s71","s73","s76","s77","s78","s79","s80","s84","scc");
  float s = acc0 + acc1 + acc2 + acc3 + acc4 + acc5 + acc6 + acc7;
  if (s == 1234.5f) out[threadIdx.x] = s;
}


__global__ void __launch_bounds__(256) fall_body_only(float* out, int iters) {
  extern __shared__ float sm[];
  for (int i = threadIdx.x; i < 4096; i += 256) sm[i] = i * 0.5f;
  __syncthreads();
  float acc0 = threadIdx.x, acc1 = 1, acc2 = 2, acc3 = 3, acc4 = 4, acc5 = 5, acc6 = 6, acc7 = 7;
  unsigned lane = threadIdx.x & 63, la = (threadIdx.x & 63) * 16;
  asm volatile("s_getpc_b64 s[68:69]\n.Lpc%=:\ns_add_u32 s68, s68, .Ltbl%=-.Lpc%=\ns_addc_u32 s69, s69, 0\ns_mov_b32 s71, s69\nv_and_b32 v41, 3, v43\nv_add_u32 v41, 1, v41\nv_and_b32 v41, 3, v41\nv_lshlrev_b32 v40, 2, v41\nv_add_u32 v40, s68, v40\nv_mov_b32 v44, v41\ns_mov_b32 s66, 0\ns_mov_b32 s84, 0\ns_mov_b32 s80, %[it]\ns_nop 4\nv_readlane_b32 s70, v40, 3\ns_nop 4\ns_branch .Lh0%=\n.Ltbl%=:\ns_branch .Lh0%=\ns_branch .Lh1%=\ns_branch .Lh2%=\ns_branch .Lh3%=\n.Lh0%=:\nv_add_f32 v32, v32, v56\nv_add_f32 v33, v33, v57\nv_add_f32 v34, v34, v58\nv_add_f32 v35, v35, v59\nv_add_f32 v36, v36, v60\nv_add_f32 v37, v37, v61\nv_add_f32 v38, v38, v62\nv_add_f32 v39, v39, v63\n.Lh1%=:\nv_add_f32 v32, v32, v48\nv_add_f32 v33, v33, v49\nv_add_f32 v34, v34, v50\nv_add_f32 v35, v35, v51\nv_add_f32 v36, v36, v52\nv_add_f32 v37, v37, v53\nv_add_f32 v38, v38, v54\nv_add_f32 v39, v39, v55\n.Lh2%=:\nv_add_f32 v32, v32, v56\nv_add_f32 v33, v33, v57\nv_add_f32 v34, v34, v58\nv_add_f32 v35, v35, v59\nv_add_f32 v36, v36, v60\nv_add_f32 v37, v37, v61\nv_add_f32 v38, v38, v62\nv_add_f32 v39, v39, v63\n.Lh3%=:\nv_add_f32 v32, v32, v48\nv_add_f32 v33, v33, v49\nv_add_f32 v34, v34, v50\nv_add_f32 v35, v35, v51\nv_add_f32 v36, v36, v52\nv_add_f32 v37, v37, v53\nv_add_f32 v38, v38, v54\nv_add_f32 v39, v39, v55\ns_sub_u32 s80, s80, 1\ns_cbranch_scc1 .Ldone%=\ns_branch .Lh0%=\n.Ldone%=:\ns_waitcnt lgkmcnt(0)" : "+{v32}"(acc0), "+{v33}"(acc1), "+{v34}"(acc2), "+{v35}"(acc3), "+{v36}"(acc4), "+{v37}"(acc5), "+{v38}"(acc6), "+{v39}"(acc7)
     : "{v43}"(lane), [it] "s"(iters), "{v42}"(la), "{s[82:83]}"(out) : "v0","v40","v41","v44","v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63","s65","s66","s68","s69","s70","s71","s73","s76","s77","s78","s79","s80","s84","scc");
  float s = acc0 + acc1 + acc2 + acc3 + acc4 + acc5 + acc6 + acc7;
  if (s == 1234.5f) out[threadIdx.x] = s;
}


__global__ void __launch_bounds__(256) rl_nolds_fall(float* out, int iters) {
  extern __shared__ float sm[];
  for (int i = threadIdx.x; i < 4096; i += 256) sm[i] = i * 0.5f;
  __syncthreads();
  float acc0 = threadIdx.x, acc1 = 1, acc2 = 2, acc3 = 3, acc4 = 4, acc5 = 5, acc6 = 6, acc7 = 7;
  unsigned lane = threadIdx.x & 63, la = (threadIdx.x & 63) * 16;
  asm volatile("s_getpc_b64 s[68:69]\n.Lpc%=:\ns_add_u32 s68, s68, .Ltbl%=-.Lpc%=\ns_addc_u32 s69, s69, 0\ns_mov_b32 s71, s69\nv_and_b32 v41, 3, v43\nv_add_u32 v41, 1, v41\nv_and_b32 v41, 3, v41\nv_lshlrev_b32 v40, 2, v41\nv_add_u32 v40, s68, v40\nv_mov_b32 v44, v41\ns_mov_b32 s66, 0\ns_mov_b32 s84, 0\ns_mov_b32 s80, %[it]\ns_nop 4\nv_readlane_b32 s70, v40, 3\ns_nop 4\ns_branch .Lh0%=\n.Ltbl%=:\ns_branch .Lh0%=\ns_branch .Lh1%=\ns_branch .Lh2%=\ns_branch .Lh3%=\n.Lh0%=:\nv_readlane_b32 s73, v42, s66\nv_readlane_b32 s70, v40, s66\nv_readlane_b32 s65, v42, s66\nv_readlane_b32 s66, v44, s66\nv_add_f32 v32, v32, v56\nv_add_f32 v33, v33, v57\nv_add_f32 v34, v34, v58\nv_add_f32 v35, v35, v59\nv_add_f32 v36, v36, v60\nv_add_f32 v37, v37, v61\nv_add_f32 v38, v38, v62\nv_add_f32 v39, v39, v63\n.Lh1%=:\nv_readlane_b32 s73, v42, s66\nv_readlane_b32 s70, v40, s66\nv_readlane_b32 s65, v42, s66\nv_readlane_b32 s66, v44, s66\nv_add_f32 v32, v32, v48\nv_add_f32 v33, v33, v49\nv_add_f32 v34, v34, v50\nv_add_f32 v35, v35, v51\nv_add_f32 v36, v36, v52\nv_add_f32 v37, v37, v53\nv_add_f32 v38, v38, v54\nv_add_f32 v39, v39, v55\n.Lh2%=:\nv_readlane_b32 s73, v42, s66\nv_readlane_b32 s70, v40, s66\nv_readlane_b32 s65, v42, s66\nv_readlane_b32 s66, v44, s66\nv_add_f32 v32, v32, v56\nv_add_f32 v33, v33, v57\nv_add_f32 v34, v34, v58\nv_add_f32 v35, v35, v59\nv_add_f32 v36, v36, v60\nv_add_f32 v37, v37, v61\nv_add_f32 v38, v38, v62\nv_add_f32 v39, v39, v63\n.Lh3%=:\nv_readlane_b32 s73, v42, s66\nv_readlane_b32 s70, v40, s66\nv_readlane_b32 s65, v42, s66\nv_readlane_b32 s66, v44, s66\nv_add_f32 v32, v32, v48\nv_add_f32 v33, v33, v49\nv_add_f32 v34, v34, v50\nv_add_f32 v35, v35, v51\nv_add_f32 v36, v36, v52\nv_add_f32 v37, v37, v53\nv_add_f32 v38, v38, v54\nv_add_f32 v39, v39, v55\ns_sub_u32 s80, s80, 1\ns_cbranch_scc1 .Ldone%=\ns_branch .Lh0%=\n.Ldone%=:\ns_waitcnt lgkmcnt(0)" : "+{v32}"(acc0), "+{v33}"(acc1), "+{v34}"(acc2), "+{v35}"(acc3), "+{v36}"(acc4), "+{v37}"(acc5), "+{v38}"(acc6), "+{v39}"(acc7)
     : "{v43}"(lane), [it] "s"(iters), "{v42}"(la), "{s[82:83]}"(out) : "v0","v40","v41","v44","v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63","s65","s66","s68","s69","s70","s71","s73","s76","s77","s78","s79","s80","s84","scc");
  float s = acc0 + acc1 + acc2 + acc3 + acc4 + acc5 + acc6 + acc7;
  if (s == 1234.5f) out[threadIdx.x] = s;
}


__global__ void __launch_bounds__(256) lds_fall(float* out, int iters) {
  extern __shared__ float sm[];
  for (int i = threadIdx.x; i < 4096; i += 256) sm[i] = i * 0.5f;
  __syncthreads();
  float acc0 = threadIdx.x, acc1 = 1, acc2 = 2, acc3 = 3, acc4 = 4, acc5 = 5, acc6 = 6, acc7 = 7;
  unsigned lane = threadIdx.x & 63, la = (threadIdx.x & 63) * 16;
  asm volatile("s_getpc_b64 s[68:69]\n.Lpc%=:\ns_add_u32 s68, s68, .Ltbl%=-.Lpc%=\ns_addc_u32 s69, s69, 0\ns_mov_b32 s71, s69\nv_and_b32 v41, 3, v43\nv_add_u32 v41, 1, v41\nv_and_b32 v41, 3, v41\nv_lshlrev_b32 v40, 2, v41\nv_add_u32 v40, s68, v40\nv_mov_b32 v44, v41\ns_mov_b32 s66, 0\ns_mov_b32 s84, 0\ns_mov_b32 s80, %[it]\ns_nop 4\nv_readlane_b32 s70, v40, 3\ns_nop 4\ns_branch .Lh0%=\n.Ltbl%=:\ns_branch .Lh0%=\ns_branch .Lh1%=\ns_branch .Lh2%=\ns_branch .Lh3%=\n.Lh0%=:\nv_add_u32 v0, 0, v42\nds_read_b128 v[48:51], v0\nds_read_b128 v[52:55], v0 offset:1024\ns_waitcnt lgkmcnt(2)\nv_add_f32 v32, v32, v56\nv_add_f32 v33, v33, v57\nv_add_f32 v34, v34, v58\nv_add_f32 v35, v35, v59\nv_add_f32 v36, v36, v60\nv_add_f32 v37, v37, v61\nv_add_f32 v38, v38, v62\nv_add_f32 v39, v39, v63\n.Lh1%=:\nv_add_u32 v0, 0, v42\nds_read_b128 v[56:59], v0\nds_read_b128 v[60:63], v0 offset:1024\ns_waitcnt lgkmcnt(2)\nv_add_f32 v32, v32, v48\nv_add_f32 v33, v33, v49\nv_add_f32 v34, v34, v50\nv_add_f32 v35, v35, v51\nv_add_f32 v36, v36, v52\nv_add_f32 v37, v37, v53\nv_add_f32 v38, v38, v54\nv_add_f32 v39, v39, v55\n.Lh2%=:\nv_add_u32 v0, 0, v42\nds_read_b128 v[48:51], v0\nds_read_b128 v[52:55], v0 offset:1024\ns_waitcnt lgkmcnt(2)\nv_add_f32 v32, v32, v56\nv_add_f32 v33, v33, v57\nv_add_f32 v34, v34, v58\nv_add_f32 v35, v35, v59\nv_add_f32 v36, v36, v60\nv_add_f32 v37, v37, v61\nv_add_f32 v38, v38, v62\nv_add_f32 v39, v39, v63\n.Lh3%=:\nv_add_u32 v0, 0, v42\nds_read_b128 v[56:59], v0\nds_read_b128 v[60:63], v0 offset:1024\ns_waitcnt lgkmcnt(2)\nv_add_f32 v32, v32, v48\nv_add_f32 v33, v33, v49\nv_add_f32 v34, v34, v50\nv_add_f32 v35, v35, v51\nv_add_f32 v36, v36, v52\nv_add_f32 v37, v37, v53\nv_add_f32 v38, v38, v54\nv_add_f32 v39, v39, v55\ns_sub_u32 s80, s80, 1\ns_cbranch_scc1 .Ldone%=\ns_branch .Lh0%=\n.Ldone%=:\ns_waitcnt lgkmcnt(0)" : "+{v32}"(acc0), "+{v33}"(acc1), "+{v34}"(acc2), "+{v35}"(acc3), "+{v36}"(acc4), "+{v37}"(acc5), "+{v38}"(acc6), "+{v39}"(acc7)
     : "{v43}"(lane), [it] "s"(iters), "{v42}"(la), "{s[82:83]}"(out) : "v0","v40","v41","v44","v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63","s65","s66","s68","s69","s70","s71","s73","s76","s77","s78","s79","s80","s84","scc");
  float s = acc0 + acc1 + acc2 + acc3 + acc4 + acc5 + acc6 + acc7;
  if (s == 1234.5f) out[threadIdx.x] = s;
}


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
  printf("%-20s occ=%d  %8.1f cyc/dispatch/SIMD  (%7.1f per wave-dispatch)\n", name, occ, cyc, cyc / occ);
}
int main() {
  float* d; CHECK(hipMalloc(&d, 4096));
  for (int occ : {1, 2, 4, 8}) {
    run("rl1_fall", rl1_fall, d, occ);
    run("rl2_fall", rl2_fall, d, occ);
    run("rlconst4_fall", rlconst4_fall, d, occ);
    run("smem_fall", smem_fall, d, occ);
    run("smem_lds_fall", smem_lds_fall, d, occ);
    run("salu4_fall", salu4_fall, d, occ);
    run("full_table", full_table, d, occ);
    run("full_direct", full_direct, d, occ);
    run("nolds_table", nolds_table, d, occ);
    run("nolds_direct", nolds_direct, d, occ);
    run("norl_nolds_direct", norl_nolds_direct, d, occ);
    run("fall_body_only", fall_body_only, d, occ);
    run("rl_nolds_fall", rl_nolds_fall, d, occ);
    run("lds_fall", lds_fall, d, occ);
  }
  CHECK(hipFree(d));
  return 0;
}
