// Device idle between two kernels on one stream with an event record, a
// cross-stream wait, or nothing between them (diagnostic; run under
// rocprofv3 --kernel-trace and read the gaps with tools/event_gap.py).
//   hipcc --offload-arch=gfx950 -O2 -o tools/_event_gap tools/event_gap.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_spin(unsigned long long ticks, int* out) {
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) {
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = 1;
}
// as k_spin, then block 0 stores the flag (after its own spin: the other
// blocks may still be running; only the gap is of interest here)
__global__ void k_spin_flag(unsigned long long ticks, int* out, uint64_t* flag, uint64_t v) {
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) {
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    out[0] = 1;
    __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
__global__ void k_mark(int* out, int v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) out[1] = v;
}

int main() {
  int* d = nullptr;
  uint64_t* flag = nullptr;
  if (hipMalloc(&d, 64) != hipSuccess) return 1;
  if (hipMalloc(&flag, 64) != hipSuccess) return 1;
  hipMemset(flag, 0, 64);
  hipStream_t s1, s2;
  hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  hipEvent_t e_dev, e_def, e_t;
  hipEventCreateWithFlags(&e_dev, hipEventDisableTiming | hipEventDisableSystemFence);
  hipEventCreateWithFlags(&e_def, hipEventDisableTiming);
  hipEventCreate(&e_t);
  const unsigned long long ticks = 2000;  // 20 us of spin at 100 MHz
  for (int rep = 0; rep < 20; ++rep) {
    // mode 1: back to back
    hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, s1, ticks, d);
    hipLaunchKernelGGL(k_mark, dim3(1), dim3(64), 0, s1, d, 1);
    // mode 2: device-scope event record between
    hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, s1, ticks, d);
    hipEventRecord(e_dev, s1);
    hipLaunchKernelGGL(k_mark, dim3(1), dim3(64), 0, s1, d, 2);
    // mode 3: default (system-fence) event record between
    hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, s1, ticks, d);
    hipEventRecord(e_def, s1);
    hipLaunchKernelGGL(k_mark, dim3(1), dim3(64), 0, s1, d, 3);
    // mode 4: a wait on an event of the same stream, already recorded
    hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, s1, ticks, d);
    hipEventRecord(e_dev, s1);
    hipStreamWaitEvent(s1, e_dev, 0);
    hipLaunchKernelGGL(k_mark, dim3(1), dim3(64), 0, s1, d, 4);
    // mode 5: cross-stream: spin on s1, record, s2 waits, mark on s2
    hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, s1, ticks, d);
    hipEventRecord(e_dev, s1);
    hipStreamWaitEvent(s2, e_dev, 0);
    hipLaunchKernelGGL(k_mark, dim3(1), dim3(64), 0, s2, d, 5);
    hipStreamSynchronize(s2);
    // mode 6: cross-stream wait on an event completed long ago
    hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, s1, ticks, d);
    hipEventRecord(e_dev, s1);
    hipStreamSynchronize(s1);
    hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, s2, ticks, d);
    hipStreamWaitEvent(s2, e_dev, 0);
    hipLaunchKernelGGL(k_mark, dim3(1), dim3(64), 0, s2, d, 6);
    // mode 7: timing event (hipEventCreate default) between
    hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, s1, ticks, d);
    hipEventRecord(e_t, s1);
    hipLaunchKernelGGL(k_mark, dim3(1), dim3(64), 0, s1, d, 7);
    hipDeviceSynchronize();
    // mode 8: a stream write-value packet between two kernels of one stream
    const uint64_t v = 100 + rep;
    hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, s1, ticks, d);
    hipStreamWriteValue64(s1, flag, v, 0);
    hipLaunchKernelGGL(k_mark, dim3(1), dim3(64), 0, s1, d, 8);
    hipDeviceSynchronize();
    // mode 9: write-value on s1 after the spin, wait-value on s2
    hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, s1, ticks, d);
    hipStreamWriteValue64(s1, flag, v + 1000, 0);
    hipStreamWaitValue64(s2, flag, v + 1000, hipStreamWaitValueGte, ~0ull);
    hipLaunchKernelGGL(k_mark, dim3(1), dim3(64), 0, s2, d, 9);
    hipDeviceSynchronize();
    // mode 10: the spin kernel stores the flag itself, s2 waits for it
    hipLaunchKernelGGL(k_spin_flag, dim3(256), dim3(256), 0, s1, ticks, d, flag, v + 2000);
    hipStreamWaitValue64(s2, flag, v + 2000, hipStreamWaitValueGte, ~0ull);
    hipLaunchKernelGGL(k_mark, dim3(1), dim3(64), 0, s2, d, 10);
    hipDeviceSynchronize();
  }
  printf("done\n");
  return 0;
}
