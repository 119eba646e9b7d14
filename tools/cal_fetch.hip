// cal_fetch.hip — calibration of rocprofv3's FETCH_SIZE / TCC request counters
// for the access shape of the summary walk (k_get_sum): independent random
// small reads, one per 128 B line.
//
// MI355X_MICROARCH.md §HBM calibrates FETCH_SIZE only for wide streaming
// reads (it reports half the bytes there) and says other widths must be
// calibrated on a known count.  Every kernel below issues a KNOWN number of
// random reads, each to a distinct 128 B line chosen by a hash:
//   k_rand<R, W, B>  : R reads per lane of W bytes (W = 16: one dwordx4; W = 64:
//                      four dwordx4 loads of one line, the summary line's shape)
//                      over a buffer of B = 0 (16 GiB, HBM-resident) or B = 1
//                      (64 MiB, Infinity-Cache resident once warm)
//   k_mix            : the summary walk's three requests (directory entry,
//                      summary line, entry) as independent reads
// The launch is repeated (a cold one, then 3 timed ones), so a PMC pass sees
// each kernel name 4 times; tools/fold_c2.py divides the counters of the
// warm launches by the known read count.  Prints reads/s per kernel (the
// random-request ceiling of bench.py's request roofline).
// build: hipcc --offload-arch=gfx950 -O3 -o tools/_build/cal_fetch tools/cal_fetch.hip
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

template <int R, int W, int B>
__global__ __launch_bounds__(256) void k_rand(const uint4* buf, uint64_t lines, uint64_t n,
                                              uint64_t salt, uint32_t* sink) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t acc = 0;
  uint4 v[R][W / 16];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint64_t line = mix((i * 8 + r) ^ salt) % lines;
#pragma unroll
    for (int w = 0; w < W / 16; ++w) v[r][w] = buf[line * 8 + w];
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int w = 0; w < W / 16; ++w) acc += v[r][w].x ^ v[r][w].w;
  if (acc == 0x12345678u) atomicAdd(sink, 1u);
}

// The summary walk's request mix as independent reads: per lane one random
// 16 B read in a 64 MiB region (the leaf directory), one random 64 B line
// in a 128 MiB region (the leaf summaries) and one random 16 B read in a
// 2 GiB region (the entries), three requests per lane (the walk's own three
// are dependent; here they are all in flight at once: the ceiling).
__global__ __launch_bounds__(256) void k_mix(const uint4* buf, uint64_t n, uint64_t salt,
                                             uint32_t* sink) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t dl = (64ull << 20) / 128, sl = (128ull << 20) / 128, el = (2ull << 30) / 128;
  const uint4* dir = buf;
  const uint4* sum = buf + (64ull << 20) / 16;
  const uint4* ent = buf + (192ull << 20) / 16;
  const uint4 a = dir[(mix(i * 3 ^ salt) % dl) * 8];
  const uint64_t sline = mix(i * 3 + 1 ^ salt) % sl;
  const uint4 b0 = sum[sline * 8], b1 = sum[sline * 8 + 1], b2 = sum[sline * 8 + 2],
              b3 = sum[sline * 8 + 3];
  const uint4 c = ent[(mix(i * 3 + 2 ^ salt) % el) * 8];
  const uint32_t acc = a.x ^ b0.y ^ b1.z ^ b2.w ^ b3.x ^ c.y;
  if (acc == 0x12345678u) atomicAdd(sink, 1u);
}

// k_mix with G independent gets' worth of requests per lane (3 G in flight)
template <int G>
__global__ __launch_bounds__(256) void k_mixg(const uint4* buf, uint64_t n, uint64_t salt,
                                              uint32_t* sink) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t dl = (64ull << 20) / 128, sl = (128ull << 20) / 128, el = (2ull << 30) / 128;
  const uint4* dir = buf;
  const uint4* sum = buf + (64ull << 20) / 16;
  const uint4* ent = buf + (192ull << 20) / 16;
  uint4 a[G], b[G][4], c[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const uint64_t j = i * G + g;
    a[g] = dir[(mix(j * 3 ^ salt) % dl) * 8];
    const uint64_t sline = mix(j * 3 + 1 ^ salt) % sl;
#pragma unroll
    for (int w = 0; w < 4; ++w) b[g][w] = sum[sline * 8 + w];
    c[g] = ent[(mix(j * 3 + 2 ^ salt) % el) * 8];
  }
  uint32_t acc = 0;
#pragma unroll
  for (int g = 0; g < G; ++g) acc ^= a[g].x ^ b[g][0].y ^ b[g][1].z ^ b[g][2].w ^ b[g][3].x ^ c[g].y;
  if (acc == 0x12345678u) atomicAdd(sink, 1u);
}

// the walk's dependent chain: directory entry -> summary line -> entry, each
// address derived from the previous load's data (the buffer holds a hash
// pattern, so the chain stays random), one chain per lane
__global__ __launch_bounds__(256) void k_chain(const uint4* buf, uint64_t n, uint64_t salt,
                                               uint32_t* sink) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t dl = (64ull << 20) / 128, sl = (128ull << 20) / 128, el = (2ull << 30) / 128;
  const uint4* dir = buf;
  const uint4* sum = buf + (64ull << 20) / 16;
  const uint4* ent = buf + (192ull << 20) / 16;
  const uint4 a = dir[(mix(i ^ salt) % dl) * 8];
  const uint64_t sline = mix(i ^ ((uint64_t)a.x << 32) ^ a.y) % sl;
  const uint4 b0 = sum[sline * 8], b1 = sum[sline * 8 + 1], b2 = sum[sline * 8 + 2],
              b3 = sum[sline * 8 + 3];
  const uint64_t eline = mix(i ^ ((uint64_t)(b0.x ^ b3.w) << 32) ^ b1.y ^ b2.z) % el;
  const uint4 c = ent[eline * 8];
  if ((c.x ^ c.y) == 0x12345678u) atomicAdd(sink, 1u);
}

__global__ void k_fill_hash(uint4* buf, uint64_t n16) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t h = mix(i);
    buf[i] = make_uint4((uint32_t)h, (uint32_t)(h >> 32), (uint32_t)(h * 3), (uint32_t)(h >> 7));
  }
}

template <class F>
void timed(const char* name, double reads, int bytes, uint64_t buffer, F launch) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  // cold launch (also warms a MALL-sized buffer), then 3 timed launches with
  // fresh addresses each (salt), so no launch re-reads the previous lines
  launch(0ull);
  CK(hipDeviceSynchronize());
  float tot = 0.f;
  for (int rep = 1; rep <= 3; ++rep) {
    CK(hipEventRecord(a));
    launch((uint64_t)rep * 0x9E3779B97F4A7C15ull);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    tot += ms;
  }
  const double ms = tot / 3;
  printf("{\"kernel\": \"%s\", \"reads_per_launch\": %.0f, \"bytes_per_read\": %d, "
         "\"buffer_bytes\": %llu, \"us\": %.2f, \"G_reads_per_s\": %.2f}\n",
         name, reads, bytes, (unsigned long long)buffer, ms * 1e3, reads / (ms * 1e-3) / 1e9);
  fflush(stdout);
}

template <int R, int W, int B>
void run(const uint4* buf, uint64_t lines, uint64_t n, uint32_t* sink, const char* name) {
  const dim3 g((unsigned)((n + 255) / 256));
  timed(name, (double)n * R, W, lines * 128, [&](uint64_t salt) {
    k_rand<R, W, B><<<g, 256>>>(buf, lines, n, salt, sink);
  });
}

int main() {
  // 16 GiB: random lines hit the 256 MiB Infinity Cache ~1.6 % of the time
  const uint64_t big = 16ull << 30, small = 64ull << 20;
  uint4* buf;
  uint32_t* sink;
  CK(hipMalloc(&buf, big));
  CK(hipMemset(buf, 1, big));
  CK(hipMalloc(&sink, 4));
  // 16 Mi lanes per launch (1-2 ms): the steady-state rate, ramp and tail
  // amortised (a 1 Mi-lane launch lasts about as long as one get walk)
  const uint64_t n = 16ull << 20, ns = 1ull << 20;
  run<4, 16, 0>(buf, big / 128, n, sink, "k_rand<4,16,0> 16GiB 16B");
  run<3, 16, 0>(buf, big / 128, n, sink, "k_rand<3,16,0> 16GiB 16B");
  run<1, 64, 0>(buf, big / 128, n, sink, "k_rand<1,64,0> 16GiB 64B");
  run<4, 16, 1>(buf, small / 128, n, sink, "k_rand<4,16,1> 64MiB 16B");
  run<1, 64, 1>(buf, small / 128, n, sink, "k_rand<1,64,1> 64MiB 64B");
  run<3, 16, 2>(buf, big / 128, ns, sink, "k_rand<3,16,2> 16GiB 16B short");
  // more reads in flight per lane, and an Infinity-Cache-sized region
  run<8, 16, 1>(buf, small / 128, n, sink, "k_rand<8,16,1> 64MiB 16B");
  run<4, 16, 3>(buf, (192ull << 20) / 128, n, sink, "k_rand<4,16,3> 192MiB 16B");
  run<4, 16, 4>(buf, (2ull << 30) / 128, n, sink, "k_rand<4,16,4> 2GiB 16B");
  const dim3 g((unsigned)((n + 255) / 256));
  timed("k_mix dir64M+sum128M(64B)+ent2G", (double)n * 3, 0, (2ull << 30) + (192ull << 20),
        [&](uint64_t salt) { k_mix<<<g, 256>>>(buf, n, salt, sink); });
  const dim3 g2((unsigned)((n / 2 + 255) / 256)), g4((unsigned)((n / 4 + 255) / 256));
  timed("k_mixg<2> dir64M+sum128M(64B)+ent2G", (double)n * 3, 0, (2ull << 30) + (192ull << 20),
        [&](uint64_t salt) { k_mixg<2><<<g2, 256>>>(buf, n / 2, salt, sink); });
  timed("k_mixg<4> dir64M+sum128M(64B)+ent2G", (double)n * 3, 0, (2ull << 30) + (192ull << 20),
        [&](uint64_t salt) { k_mixg<4><<<g4, 256>>>(buf, n / 4, salt, sink); });
  // the dependent chain reads hash data: fill the walk's regions first
  k_fill_hash<<<4096, 256>>>(buf, ((2ull << 30) + (192ull << 20)) / 16);
  CK(hipDeviceSynchronize());
  timed("k_chain dir64M->sum128M(64B)->ent2G", (double)n * 3, 0, (2ull << 30) + (192ull << 20),
        [&](uint64_t salt) { k_chain<<<g, 256>>>(buf, n, salt, sink); });
  timed("k_chain short 1Mi lanes", (double)ns * 3, 0, (2ull << 30) + (192ull << 20),
        [&](uint64_t salt) { k_chain<<<dim3((unsigned)((ns + 255) / 256)), 256>>>(buf, ns, salt, sink); });
  return 0;
}
