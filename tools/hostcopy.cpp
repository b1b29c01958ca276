// Host copy throughput into fresh vs touched memory (the per-row output
// staging of srhip_eval_tree_array, api.cpp copy_rows_to_host): 0.82 GB in
// 48 MB chunks on 1-32 threads. Build: g++ -O2 -pthread tools/hostcopy.cpp -o tools/hostcopy
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>
#include <sys/mman.h>
int main(int argc, char** argv) {
  const size_t N = 819200000ull, H = 48ull << 20;
  std::vector<unsigned char> src(2 * H, 1);
  for (int nthr : {1, 8, 16, 32}) {
    for (int touch = 0; touch < 2; ++touch) {
      unsigned char* dst = (unsigned char*)malloc(N);
      if (touch) memset(dst, 0, N);
      auto t0 = std::chrono::steady_clock::now();
      for (size_t off = 0; off < N; off += H) {
        size_t n = std::min(H, N - off);
        std::vector<std::thread> th;
        size_t per = (n + nthr - 1) / nthr;
        for (int j = 0; j < nthr; ++j) {
          size_t b = j * per, e = std::min(n, b + per);
          if (b < e) th.emplace_back([=, &src] { memcpy(dst + off + b, src.data() + ((off / H) & 1) * H + b, e - b); });
        }
        for (auto& t : th) t.join();
      }
      double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      printf("threads %d prefaulted %d: %.1f ms, %.1f GB/s\n", nthr, touch, s * 1e3, N / s / 1e9);
      free(dst);
    }
  }
}
