// ms_lines.hip — microbenchmark: how many random small reads per second HBM
// serves (the question behind a fingerprint-side-array get walk: ~5 random
// 16 B reads per get, two dependent, against one 1 KB page DMA per get).
// Each lane issues R independent random 16 B loads (distinct 128 B lines of a
// 2 GiB buffer), then, with DEP, one more load at an address taken from the
// first load's data.  Prints reads/s and GB/s of 128 B lines touched.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/_build/ms_lines tools/ms_lines.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));               \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

template <int R, bool DEP>
__global__ __launch_bounds__(256) void k_lines(const uint4* buf, uint64_t lines, uint64_t n,
                                               uint32_t* sink) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint4 v[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint64_t line = mix(i * 8 + r) % lines;
    v[r] = buf[line * 8];  // 16 B at the start of a 128 B line
  }
  uint32_t acc = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) acc += v[r].x ^ v[r].w;
  if (DEP) {
    const uint64_t line = mix(acc + i) % lines;
    const uint4 w = buf[line * 8 + 2];
    acc += w.y;
  }
  if (acc == 0x12345678u) atomicAdd(sink, 1u);
}

template <int R, bool DEP>
float run(const uint4* buf, uint64_t lines, uint64_t n, uint32_t* sink) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const dim3 g((unsigned)((n + 255) / 256));
  k_lines<R, DEP><<<g, 256>>>(buf, lines, n, sink);
  CK(hipDeviceSynchronize());
  float best = 1e9f;
  for (int rep = 0; rep < 5; ++rep) {
    CK(hipEventRecord(a));
    k_lines<R, DEP><<<g, 256>>>(buf, lines, n, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    best = ms < best ? ms : best;
  }
  return best;
}

int main() {
  const uint64_t bytes = 2ull << 30, lines = bytes / 128;
  uint4* buf;
  uint32_t* sink;
  CK(hipMalloc(&buf, bytes));
  CK(hipMemset(buf, 1, bytes));
  CK(hipMalloc(&sink, 4));
  const uint64_t n = 1 << 20;  // "queries"
  struct V {
    const char* name;
    int reads;
    float (*f)(const uint4*, uint64_t, uint64_t, uint32_t*);
  } vs[] = {{"R1", 1, run<1, false>},          {"R2", 2, run<2, false>},
            {"R4", 4, run<4, false>},          {"R4 + 1 dependent", 5, run<4, true>},
            {"R3 + 1 dependent", 4, run<3, true>}, {"R8", 8, run<8, false>}};
  for (auto& v : vs) {
    const float ms = v.f(buf, lines, n, sink);
    const double reads = (double)n * v.reads;
    printf("%-18s %8.1f us  %6.1f G reads/s  %7.1f GB/s of 128 B lines  %6.1f us per 1 Mi gets\n",
           v.name, ms * 1e3, reads / (ms * 1e-3) / 1e9, reads * 128 / (ms * 1e-3) / 1e9, ms * 1e3);
  }
  return 0;
}
