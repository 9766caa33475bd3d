// Probe: which parts of a raw buffer load's offset does gfx950's range check cover?
//
// A descriptor over the first 256 bytes of a 4 MiB buffer filled with 0x5A5A5A5A; lane 0 loads
//   (a) voffset 4096, soffset 0          -> 0 if the VGPR offset is range-checked
//   (b) voffset 0, immediate offset 1024 -> 0 if the immediate offset is range-checked
//   (c) voffset 0, soffset 4096 (SGPR)   -> 0 if the SGPR offset is range-checked
//   (d) voffset 0, soffset 0             -> 0x5A5A5A5A (in range, control)
// Every address stays inside the 4 MiB allocation, so no outcome can fault.  Used to decide
// whether a strided load may carry its stride in soffset (ppr.hip load_head, score.hip chunks).
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void probe(const unsigned* buf, unsigned soff, unsigned* out) {
  if (threadIdx.x != 0) return;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned*>(buf), 0, 256, 0x00020000);
  const unsigned v = __builtin_amdgcn_readfirstlane(soff);  // an SGPR value the compiler cannot fold
  out[0] = __builtin_amdgcn_raw_buffer_load_b32(rs, 4096 + (int)threadIdx.x, 0, 0);
  out[1] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)threadIdx.x + 1024, 0, 0);
  out[2] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)threadIdx.x, (int)v, 0);
  out[3] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)threadIdx.x, 0, 0);
}

int main() {
  unsigned *buf = nullptr, *out = nullptr;
  const size_t n = 1u << 20;
  if (hipMalloc(&buf, n * 4) != hipSuccess || hipMalloc(&out, 16) != hipSuccess) return 2;
  (void)hipMemset(buf, 0x5A, n * 4);
  (void)hipMemset(out, 0xFF, 16);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, buf, 4096u, out);
  unsigned h[4];
  if (hipMemcpy(h, out, 16, hipMemcpyDeviceToHost) != hipSuccess) return 3;
  const char* name[4] = {"voffset 4096", "imm offset 1024", "soffset 4096", "in range"};
  for (int i = 0; i < 4; ++i) printf("%-16s -> 0x%08x (%s)\n", name[i], h[i], h[i] ? "read memory" : "returned 0");
  printf("sgpr_offset_range_checked=%d\n", h[2] == 0 ? 1 : 0);
  return 0;
}
