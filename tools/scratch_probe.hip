// Dispatch cost of kernels with a private (scratch) segment on this runtime:
// an idle-work kernel whose lanes own a private array (forced to scratch by
// a dynamic index), timed with events against the same kernel without it,
// each call after a host sync (like the library's blocking calls).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int N>
__global__ void probe(const int* flag, int* out) {
  volatile int buf[N];
  const int t = threadIdx.x;
  if (*flag) {  // never true: the work is skipped, the scratch segment is not
    for (int i = 0; i < N; ++i) buf[i] = i * t;
    out[blockIdx.x * blockDim.x + t] = buf[(t * 7) % N];
  }
}

template <int N>
float run(int grid, int reps) {
  int *flag, *out;
  (void)hipMalloc(&flag, 4);
  (void)hipMemset(flag, 0, 4);
  (void)hipMalloc(&out, (size_t)grid * 256 * 4);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float best = 1e9, sum = 0;
  for (int r = 0; r < reps; ++r) {
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL(probe<N>, dim3(grid), dim3(256), 0, 0, flag, out);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    if (r) { sum += ms; best = ms < best ? ms : best; }
  }
  (void)hipFree(flag);
  (void)hipFree(out);
  printf("private %6d B/lane grid %5d: mean %.3f ms best %.3f ms\n", N * 4, grid, sum / (reps - 1), best);
  return best;
}

int main() {
  for (int grid : {1, 64, 850}) {
    run<1>(grid, 8);
    run<64>(grid, 8);
    run<400>(grid, 8);
    run<640>(grid, 8);
  }
  return 0;
}
