// FETCH_SIZE calibration for the access shapes of the PageRank step (MI355X_MICROARCH.md §HBM:
// "other access widths are uncalibrated: calibrate on a known byte count in your own access
// pattern").  Measurement tool only (not part of libkrca).  Kernels, one launch each:
//   stream16    1 GiB read as 16 B per lane, coalesced        (known: 1 GiB)
//   gather8_big 16M random 8-B reads from a 2 GiB table        (known: 16M distinct 64-B lines)
//   gather8_l3  16M random 8-B reads from an 8 MiB table       (Infinity-Cache / L2 resident)
//   gather8_run 16M 8-B reads, runs of 8 consecutive words per 8 lanes from a 2 GiB table
//               (known: 2M distinct 64-B lines; the dictionary blocks' sorted-column shape)
// Build: hipcc --offload-arch=gfx950 -O3 tools/pmc_calib.hip -o tools/bin/pmc_calib
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void stream16(const uint4* __restrict__ a, int64_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9E3779B9u) out[0] = acc;  // keep the loads
}

__global__ void gather8(const int64_t* __restrict__ t, int64_t tn, const uint32_t* __restrict__ idx, int64_t m,
                        int64_t* out) {
  int64_t acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
    acc += t[idx[i] % tn];
  if (acc == 0x123456789LL) out[0] = acc;
}

__global__ void make_idx(uint32_t* idx, int64_t m, int run, uint32_t span) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t g = (uint64_t)(i / run);
    uint64_t h = g * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 32;
    const uint32_t base = (uint32_t)(h % (span / 8)) * 8;  // 64-B aligned line start
    idx[i] = base + (uint32_t)(i % run);
  }
}

int main() {
  const int64_t big = (int64_t)1 << 28;   // 2 GiB of int64
  const int64_t small = (int64_t)1 << 20;  // 8 MiB of int64
  const int64_t m = (int64_t)1 << 24;      // 16M gathers
  int64_t* t;
  uint32_t* idx;
  int64_t* out;
  CHECK(hipMalloc(&t, big * 8));
  CHECK(hipMalloc(&idx, m * 4));
  CHECK(hipMalloc(&out, 64));
  CHECK(hipMemset(t, 1, big * 8));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  float ms;
  // stream16 over the first GiB
  (void)hipEventRecord(e0);
  stream16<<<4096, 256>>>(reinterpret_cast<const uint4*>(t), ((int64_t)1 << 30) / 16, reinterpret_cast<uint32_t*>(out));
  (void)hipEventRecord(e1);
  CHECK(hipEventSynchronize(e1));
  (void)hipEventElapsedTime(&ms, e0, e1);
  printf("{\"kernel\": \"stream16\", \"bytes\": %lld, \"ms\": %.4f}\n", (long long)1 << 30, ms);
  struct Case { const char* name; int64_t tn; int run; };
  const Case cases[3] = {{"gather8_big", big, 1}, {"gather8_l3", small, 1}, {"gather8_run", big, 8}};
  for (const Case& c : cases) {
    make_idx<<<4096, 256>>>(idx, m, c.run, (uint32_t)(c.tn > (int64_t)0xFFFFFFF8 ? 0xFFFFFFF8 : c.tn));
    CHECK(hipDeviceSynchronize());
    (void)hipEventRecord(e0);
    gather8<<<4096, 256>>>(t, c.tn, idx, m, out);
    (void)hipEventRecord(e1);
    CHECK(hipEventSynchronize(e1));
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("{\"kernel\": \"%s\", \"gathers\": %lld, \"distinct_lines_64B\": %lld, \"idx_bytes\": %lld, \"ms\": %.4f}\n",
           c.name, (long long)m, (long long)(m / c.run), (long long)(m * 4), ms);
  }
  (void)hipFree(t);
  (void)hipFree(idx);
  (void)hipFree(out);
  return 0;
}
