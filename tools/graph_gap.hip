// Per-kernel cost of dependent kernels that return at once: stream launches
// against the same chain captured in a hipGraph (diagnostic, round 5):
//   hipcc --offload-arch=gfx950 -O2 -o tools/_graph_gap tools/graph_gap.hip && tools/_graph_gap
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_nop(const unsigned* flag, unsigned* out) {
  if (*flag == 0) return;  // always
  out[blockIdx.x] = threadIdx.x;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  unsigned *flag = nullptr, *out = nullptr;
  CK(hipMalloc(&flag, 4));
  CK(hipMalloc(&out, 1 << 20));
  CK(hipMemset(flag, 0, 4));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int chain = 8, reps = 200;
  for (int grid : {1, 256, 1024}) {
    // stream launches
    for (int w = 0; w < 2; ++w) {
      CK(hipEventRecord(a, s));
      for (int r = 0; r < reps; ++r)
        for (int c = 0; c < chain; ++c) hipLaunchKernelGGL(k_nop, dim3(grid), dim3(256), 0, s, flag, out);
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
    }
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("grid %4d stream: %.2f us per kernel\n", grid, ms * 1e3 / (reps * chain));
    // one graph of `chain` kernels, launched reps times
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int c = 0; c < chain; ++c) hipLaunchKernelGGL(k_nop, dim3(grid), dim3(256), 0, s, flag, out);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int w = 0; w < 2; ++w) {
      CK(hipEventRecord(a, s));
      for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
    }
    CK(hipEventElapsedTime(&ms, a, b));
    printf("grid %4d graph : %.2f us per kernel\n", grid, ms * 1e3 / (reps * chain));
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  return 0;
}
