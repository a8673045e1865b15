// SPDX-License-Identifier: BSD-2-Clause
// Probe: after `s_waitcnt vmcnt(0)` retires a global_load_lds_dwordx4, does
// an immediate ds_read of its LDS bytes always see them?  Every wave streams
// 1-KiB pieces through a ring and checks each piece right after the wait
// that retires it.  MODE 0: read at once; 1: s_barrier between wait and read;
// 2: s_nop padding; 3: read, discard, read again; 4: ring 8 deep (counted
// vmcnt(7)).  Prints mismatching 16-B cells per mode.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __attribute__((address_space(3))) void* lptr;
typedef const __attribute__((address_space(1))) void* gptr;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 rd(const void* p) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"((uint32_t)(uintptr_t)(lptr)(p)) : "memory");
  return v;
}

template <int MODE, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void k(const u32x4* src, size_t npieces, uint32_t* bad) {
  __shared__ __attribute__((aligned(16))) u32x4 ring[WAVES][8][64];
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t gw = (size_t)blockIdx.x * WAVES + w, nw = (size_t)gridDim.x * WAVES;
  uint32_t nb = 0;
  constexpr int D = MODE == 4 ? 8 : 1;
  size_t p0 = gw;
  // prologue
  for (int u = 0; u < D; ++u) {
    const size_t p = p0 + (size_t)u * nw;
    __builtin_amdgcn_global_load_lds((gptr)(src + (p % npieces) * 64 + lane), (lptr)&ring[w][u][0], 16, 0, 2);
  }
  for (int it = 0; it < 256; ++it) {
    const int u = it % D;
    const size_t p = p0 + (size_t)it * nw;
    if (MODE == 4) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (MODE == 1) __builtin_amdgcn_s_barrier();
    if (MODE == 2) asm volatile("s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");
    u32x4 v = rd(&ring[w][u][lane]);
    if (MODE == 3) v = rd(&ring[w][u][lane]);
    const u32x4 want = src[(p % npieces) * 64 + lane];
    nb += (v.x != want.x) | (v.y != want.y) | (v.z != want.z) | (v.w != want.w);
    const size_t pn = p + (size_t)D * nw;
    __builtin_amdgcn_global_load_lds((gptr)(src + (pn % npieces) * 64 + lane), (lptr)&ring[w][u][0], 16, 0, 2);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (nb) atomicAdd(bad, nb);
}

int main() {
  const size_t npieces = (size_t)1 << 20;  // 1 GiB
  u32x4* src;
  uint32_t* bad;
  if (hipMalloc(&src, npieces * 1024) != hipSuccess || hipMalloc(&bad, 4) != hipSuccess) return 1;
  // distinct content per 16 B
  u32x4* h = (u32x4*)malloc(1 << 26);
  for (size_t off = 0; off < npieces * 64; off += (1 << 22)) {
    for (size_t i = 0; i < (1 << 22); ++i) { const uint32_t x = (uint32_t)(off + i); h[i] = (u32x4){x, x * 2654435761u, ~x, x ^ 0x5a5a5a5au}; }
    (void)hipMemcpy(src + off, h, (size_t)1 << 26, hipMemcpyHostToDevice);
  }
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int grid = prop.multiProcessorCount * 4;
  auto run = [&](auto kern, int mode) {
    (void)hipMemset(bad, 0, 4);
    for (int r = 0; r < 4; ++r) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, src, npieces, bad);
    uint32_t b = 0;
    (void)hipMemcpy(&b, bad, 4, hipMemcpyDeviceToHost);
    printf("{\"mode\":%d,\"bad_cells\":%u,\"checked_cells\":%zu}\n", mode, b, (size_t)4 * grid * 4 * 256 * 64);
  };
  run(k<0, 4>, 0);
  run(k<1, 4>, 1);
  run(k<2, 4>, 2);
  run(k<3, 4>, 3);
  run(k<4, 4>, 4);
  return 0;
}
