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

// a big kernel argument (as the library's UpperArgs, ~600 B)
struct Big {
  unsigned long long w[75];
};
template <int LDS>
__global__ __launch_bounds__(512) void k_empty_big(Big b, const unsigned* flag, unsigned* out) {
  __shared__ unsigned s[LDS / 4];
  if (*flag == 0) return;
  s[threadIdx.x % (LDS / 4)] = (unsigned)b.w[threadIdx.x % 75];
  __syncthreads();
  out[blockIdx.x] = s[(threadIdx.x + 1) % (LDS / 4)];
}
// a writer before the empty kernels (dirties L2 with 64 MB of scattered lines)
__global__ void k_write(unsigned* buf, unsigned n) {
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    buf[(i * 2654435761u) % n] = i;
}

int main() {
  unsigned *flag = nullptr, *out = nullptr;
  hipMalloc(&flag, 4);
  hipMalloc(&out, 4 << 20);
  hipMemset(flag, 0, 4);
  hipStream_t s;
  hipStreamCreate(&s);
  unsigned* wbuf = nullptr;
  hipMalloc(&wbuf, 64u << 20);
  Big big{};
  for (int rep = 0; rep < 20; ++rep) {
    hipLaunchKernelGGL(k_write, dim3(1024), dim3(256), 0, s, wbuf, (64u << 20) / 4);
    hipLaunchKernelGGL(k_empty_big<65536>, dim3(256), dim3(512), 0, s, big, flag, out);
    hipLaunchKernelGGL(k_empty_big<65536>, dim3(256), dim3(512), 0, s, big, flag, out);
    hipLaunchKernelGGL(k_empty_big<53248>, dim3(768), dim3(256), 0, s, big, flag, out);
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
