#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <fstream>
#include <vector>
#include <iterator>
int main(int argc, char** argv) {
  hipSetDevice(0);
  float* d; hipMalloc(&d, 4);
  for (int a = 1; a < argc; ++a) {
    std::ifstream f(argv[a], std::ios::binary);
    std::vector<char> img((std::istreambuf_iterator<char>(f)), {});
    double tl = 0, tr = 0, tu = 0;
    const int N = 10;
    for (int i = 0; i < N + 1; ++i) {
      auto t0 = std::chrono::steady_clock::now();
      hipModule_t m; hipFunction_t fn;
      if (hipModuleLoadData(&m, img.data()) != hipSuccess) { printf("load failed\n"); return 1; }
      if (hipModuleGetFunction(&fn, m, "sr_tmpl") != hipSuccess) { printf("getfn failed\n"); return 1; }
      auto t1 = std::chrono::steady_clock::now();
      void* args[] = {&d};
      hipModuleLaunchKernel(fn, 1, 1, 1, 64, 1, 1, 0, 0, args, nullptr);
      hipDeviceSynchronize();
      auto t2 = std::chrono::steady_clock::now();
      hipModuleUnload(m);
      auto t3 = std::chrono::steady_clock::now();
      if (i) { tl += std::chrono::duration<double, std::milli>(t1 - t0).count();
               tr += std::chrono::duration<double, std::milli>(t2 - t1).count();
               tu += std::chrono::duration<double, std::milli>(t3 - t2).count(); }
    }
    printf("%s bytes=%zu load+getfn %.3f ms  first launch %.3f ms  unload %.3f ms\n", argv[a], img.size(), tl / N, tr / N, tu / N);
  }
  return 0;
}
