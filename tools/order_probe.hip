// Stream-order probe: kernel A (many workgroups, the last ones slow) writes
// x[i] = gen; kernel B, launched next on the same stream, counts entries not
// yet equal to gen. Any nonzero count means B started before A finished.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void writer(unsigned* x, unsigned gen, int spin) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x >= gridDim.x - 64) {  // the last workgroups dawdle
    long long t0 = clock64();
    while (clock64() - t0 < spin) {}
  }
  x[i] = gen;
}
__global__ void reader(const unsigned* x, unsigned gen, unsigned n, unsigned long long* bad) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && x[i] != gen) atomicAdd(bad, 1ull);
}

int main() {
  const unsigned nb = 217344 / 256 * 256, n = nb * 256;
  unsigned* x;
  unsigned long long *bad, hb;
  (void)hipMalloc(&x, n * 4);
  (void)hipMalloc(&bad, 8);
  for (int mode = 0; mode < 2; ++mode) {
    unsigned long long total = 0;
    for (unsigned gen = 1; gen <= 20; ++gen) {
      (void)hipMemset(bad, 0, 8);
      (void)hipDeviceSynchronize();
      hipLaunchKernelGGL(writer, dim3(nb), dim3(256), 0, 0, x, gen + 100 * mode, 200000);
      if (mode == 1) (void)hipMemsetAsync(bad, 0, 8, 0);
      hipLaunchKernelGGL(reader, dim3(nb), dim3(256), 0, 0, x, gen + 100 * mode, n, bad);
      (void)hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
      total += hb;
    }
    printf("mode %d (%s): entries read before written, 20 runs: %llu\n", mode,
           mode ? "memset between" : "back to back", total);
  }
  return 0;
}
