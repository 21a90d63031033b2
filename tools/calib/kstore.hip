// Launch-cost probe: durations of tiny kernels (empty, a device-memory store, a store to
// host-mapped coherent memory, and the k_bdyval_qc shape: 23 blocks of 256 threads) under
// rocprofv3 --kernel-trace --stats.  hipcc --offload-arch=gfx950 -O3 kstore.hip -o kstore
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { if ((x) != hipSuccess) { std::printf("HIP error %s\n", #x); return 1; } } while (0)
struct Snap { int a, b; long long c; };
__global__ void k_empty() {}
__global__ void k_dev_store(const double* s, Snap* r) {
  if (threadIdx.x == 0) { const double x = s[0]; r[0].a = (int)x; r[0].c = 1; }
}
__global__ void k_host_store(const double* s, Snap* r) {
  if (threadIdx.x == 0) { const double x = s[0]; r[0].a = (int)x; r[0].c = 1; }
}
__global__ void k_blocks23(double* q) {
  const int k = blockIdx.x;
  q[k * 256 + threadIdx.x] += 1.0;
}
int main() {
  double* s; Snap *dr, *hr, *hd; double* q;
  CK(hipMalloc(&s, 64)); CK(hipMemset(s, 0, 64));
  CK(hipMalloc(&dr, 64 * sizeof(Snap)));
  CK(hipHostMalloc((void**)&hr, 64 * sizeof(Snap), hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer((void**)&hd, hr, 0));
  CK(hipMalloc(&q, 23 * 256 * sizeof(double))); CK(hipMemset(q, 0, 23 * 256 * sizeof(double)));
  hipStream_t st; CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  for (int it = 0; it < 2000; it++) {
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st);
    hipLaunchKernelGGL(k_dev_store, dim3(1), dim3(64), 0, st, s, dr);
    hipLaunchKernelGGL(k_host_store, dim3(1), dim3(64), 0, st, s, hd);
    hipLaunchKernelGGL(k_blocks23, dim3(23), dim3(256), 0, st, q);
  }
  CK(hipStreamSynchronize(st));
  std::printf("done %d\n", hr[0].a);
  return 0;
}
