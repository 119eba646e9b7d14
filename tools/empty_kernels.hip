// Duration of kernels that return at once, by grid, block and static LDS
// (diagnostic; rocprofv3 --kernel-trace --stats):
//   hipcc --offload-arch=gfx950 -O2 -o tools/_empty_kernels tools/empty_kernels.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int LDS>
__global__ void k_empty(const unsigned* flag, unsigned* out) {
  __shared__ unsigned s[LDS / 4 > 0 ? LDS / 4 : 1];
  if (*flag == 0) return;  // always: the flag is 0
  s[threadIdx.x % (LDS / 4 > 0 ? LDS / 4 : 1)] = threadIdx.x;
  __syncthreads();
  out[blockIdx.x] = s[(threadIdx.x + 1) % (LDS / 4 > 0 ? LDS / 4 : 1)];
}

int main() {
  unsigned *flag = nullptr, *out = nullptr;
  hipMalloc(&flag, 4);
  hipMalloc(&out, 4 << 20);
  hipMemset(flag, 0, 4);
  hipStream_t s;
  hipStreamCreate(&s);
  for (int rep = 0; rep < 20; ++rep) {
    hipLaunchKernelGGL(k_empty<4>, dim3(256), dim3(256), 0, s, flag, out);
    hipLaunchKernelGGL(k_empty<4>, dim3(768), dim3(256), 0, s, flag, out);
    hipLaunchKernelGGL(k_empty<4>, dim3(2048), dim3(256), 0, s, flag, out);
    hipLaunchKernelGGL(k_empty<53248>, dim3(768), dim3(256), 0, s, flag, out);
    hipLaunchKernelGGL(k_empty<65536>, dim3(256), dim3(512), 0, s, flag, out);
    hipLaunchKernelGGL(k_empty<4>, dim3(1), dim3(64), 0, s, flag, out);
  }
  hipStreamSynchronize(s);
  printf("done\n");
  return 0;
}
