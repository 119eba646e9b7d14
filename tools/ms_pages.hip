// ms_pages.hip — microbenchmark: the HBM ceiling for the get walk's access
// pattern.  Gathers N distinct random 1 KB pages of a 2 GiB arena (the leaf
// reads of one 1 Mi-query batch over the C2 tree are ~0.8 M such pages), P
// consecutive list entries per wave, D pages in flight per wave through an
// LDS-DMA ring, no page resolution (one LDS dword per page is summed so the
// data is consumed).  Prints GB/s for each (D, P, sorted) variant.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/_build/ms_pages tools/ms_pages.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#pragma clang diagnostic ignored "-Winline-asm"

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));               \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

__device__ __forceinline__ void glds16(const uint8_t* page, uint32_t lds_addr) {
  const uint64_t ga = (uint64_t)(page + 16 * __lane_id());
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(ga), "s"(lds_addr)
               : "memory", "m0");
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int D, int WPB>
__global__ __launch_bounds__(WPB * 64) void k_gather(const uint8_t* arena, const uint32_t* pages,
                                                      uint32_t n, uint32_t per_wave,
                                                      uint32_t* sink) {
  __shared__ __attribute__((aligned(16))) uint32_t ring[WPB][D][256];
  const int wv = threadIdx.x >> 6;
  const uint64_t w = (uint64_t)blockIdx.x * WPB + wv;
  const uint64_t b = w * per_wave;
  if (b >= n) return;
  const uint32_t m = (uint32_t)std::min<uint64_t>(per_wave, n - b);
  const uint32_t base = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint32_t*)&ring[wv][0][0]));
  uint32_t acc = 0;
  for (uint32_t j = 0; j < D - 1 && j < m; ++j)
    glds16(arena + (uint64_t)pages[b + j] * 1024, base + (j % D) * 1024);
  for (uint32_t j = 0; j < m; ++j) {
    if (j + D - 1 < m) {
      glds16(arena + (uint64_t)pages[b + j + D - 1] * 1024, base + ((j + D - 1) % D) * 1024);
      wait_vm<D - 1>();
    } else {
      wait_vm<0>();
    }
    acc += ring[wv][j % D][__lane_id() * 4];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// group pattern of the get walk: G DMAs per group, NB group buffers, C
// dependent VALU ops of "resolution" per group
template <int G, int NB, int WPB, int C>
__global__ __launch_bounds__(WPB * 64) void k_group(const uint8_t* arena, const uint32_t* pages,
                                                     uint32_t n, uint32_t per_wave,
                                                     uint32_t* sink) {
  __shared__ __attribute__((aligned(16))) uint32_t ring[WPB][NB][G][256];
  const int wv = threadIdx.x >> 6;
  const uint64_t w = (uint64_t)blockIdx.x * WPB + wv;
  const uint64_t b = w * per_wave;
  if (b >= n) return;
  const uint32_t m = (uint32_t)std::min<uint64_t>(per_wave, n - b);
  const uint32_t ng = (m + G - 1) / G;
  const uint32_t base = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint32_t*)&ring[wv][0][0][0]));
  auto issue = [&](uint32_t g) {
    for (int s = 0; s < G; ++s) {
      const uint32_t j = g * G + s;
      const uint32_t pg = j < m ? pages[b + j] : 0;
      glds16(arena + (uint64_t)pg * 1024, base + ((g % NB) * G + s) * 1024);
    }
  };
  uint32_t acc = __lane_id();
  for (uint32_t g = 0; g < NB && g < ng; ++g) issue(g);
  for (uint32_t g = 0; g < ng; ++g) {
    const uint32_t later = std::min<uint32_t>(NB - 1, ng - 1 - g);
    if (later >= 2) wait_vm<2 * G>();
    else if (later == 1) wait_vm<G>();
    else wait_vm<0>();
    for (int s = 0; s < G; ++s) acc += ring[wv][g % NB][s][__lane_id() * 4];
#pragma unroll
    for (int c = 0; c < C; ++c) acc = acc * 3 + (acc >> 7);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (g + NB < ng) issue(g + NB);
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int G, int NB, int WPB, int C>
float run_group(const uint8_t* arena, const uint32_t* pages, uint32_t n, uint32_t per_wave,
                uint32_t* sink) {
  const uint64_t waves = (n + per_wave - 1) / per_wave;
  dim3 grid((unsigned)((waves + WPB - 1) / WPB));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i)
    hipLaunchKernelGGL((k_group<G, NB, WPB, C>), grid, dim3(WPB * 64), 0, 0, arena, pages, n,
                       per_wave, sink);
  CK(hipEventRecord(e0, 0));
  const int reps = 20;
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL((k_group<G, NB, WPB, C>), grid, dim3(WPB * 64), 0, 0, arena, pages, n,
                       per_wave, sink);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

template <int D, int WPB>
float run(const uint8_t* arena, const uint32_t* pages, uint32_t n, uint32_t per_wave,
          uint32_t* sink) {
  const uint64_t waves = (n + per_wave - 1) / per_wave;
  dim3 grid((unsigned)((waves + WPB - 1) / WPB));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i)
    hipLaunchKernelGGL((k_gather<D, WPB>), grid, dim3(WPB * 64), 0, 0, arena, pages, n, per_wave,
                       sink);
  CK(hipEventRecord(e0, 0));
  const int reps = 20;
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL((k_gather<D, WPB>), grid, dim3(WPB * 64), 0, 0, arena, pages, n, per_wave,
                       sink);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main(int argc, char** argv) {
  const uint64_t arena_pages = 1900000;  // ~C2 tree
  const uint32_t n = argc > 1 ? atoi(argv[1]) : 800000;
  uint8_t* arena;
  CK(hipMalloc(&arena, arena_pages * 1024));
  CK(hipMemset(arena, 1, arena_pages * 1024));
  std::vector<uint32_t> all(arena_pages);
  std::iota(all.begin(), all.end(), 0u);
  std::mt19937_64 rng(7);
  std::shuffle(all.begin(), all.end(), rng);
  std::vector<uint32_t> sorted(all.begin(), all.begin() + n), rnd = sorted;
  std::sort(sorted.begin(), sorted.end());
  uint32_t *d_sorted, *d_rnd, *sink;
  CK(hipMalloc(&d_sorted, n * 4));
  CK(hipMalloc(&d_rnd, n * 4));
  CK(hipMalloc(&sink, 4));
  CK(hipMemcpy(d_sorted, sorted.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_rnd, rnd.data(), n * 4, hipMemcpyHostToDevice));
  struct VG {
    const char* name;
    float (*f)(const uint8_t*, const uint32_t*, uint32_t, uint32_t, uint32_t*);
  } gs[] = {{"G4 NB2 W4 C0", run_group<4, 2, 4, 0>},   {"G4 NB2 W4 C100", run_group<4, 2, 4, 100>},
            {"G4 NB2 W4 C300", run_group<4, 2, 4, 300>}, {"G2 NB2 W4 C0", run_group<2, 2, 4, 0>},
            {"G2 NB2 W4 C150", run_group<2, 2, 4, 150>}, {"G4 NB1 W4 C0", run_group<4, 1, 4, 0>},
            {"G2 NB3 W4 C0", run_group<2, 3, 4, 0>},     {"G1 NB4 W4 C50", run_group<1, 4, 4, 50>},
            {"G1 NB4 W4 C100", run_group<1, 4, 4, 100>}, {"G4 NB2 W1 C0", run_group<4, 2, 1, 0>}};
  for (auto& v : gs) {
    const float ms = v.f(arena, d_sorted, n, 52, sink);
    printf("%-16s per_wave 52 sorted: %.1f us  %.0f GB/s\n", v.name, ms * 1e3,
           n * 1024.0 / (ms * 1e-3) / 1e9);
  }
  if (argc > 2) return 0;
  struct V {
    const char* name;
    float (*f)(const uint8_t*, const uint32_t*, uint32_t, uint32_t, uint32_t*);
  } vs[] = {{"D2 WPB4", run<2, 4>}, {"D4 WPB4", run<4, 4>}, {"D8 WPB4", run<8, 4>},
            {"D4 WPB1", run<4, 1>}, {"D8 WPB1", run<8, 1>}, {"D16 WPB1", run<16, 1>}};
  const uint32_t pws[] = {13, 52, 208};
  for (auto& v : vs)
    for (uint32_t pw : pws)
      for (int srt = 1; srt >= 0; --srt) {
        const float ms = v.f(arena, srt ? d_sorted : d_rnd, n, pw, sink);
        printf("%-9s per_wave %3u %s: %.1f us  %.0f GB/s\n", v.name, pw, srt ? "sorted" : "random",
               ms * 1e3, n * 1024.0 / (ms * 1e-3) / 1e9);
      }
  return 0;
}
