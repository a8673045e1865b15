// SPDX-License-Identifier: BSD-2-Clause
// Probe: do ds_permute_b32 / ds_bpermute_b32 leave LDS memory untouched, and
// does either disturb LDS-DMA (global_load_lds_dwordx4) data landing at the
// same time?  Prints the number of LDS words that changed.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __attribute__((address_space(3))) void* lptr;
typedef const __attribute__((address_space(1))) void* gptr;

template <int MODE>
__global__ void k(const uint4* src, uint32_t* bad, int iters) {
  __shared__ __attribute__((aligned(16))) uint4 s[8][64];
  const uint32_t lane = threadIdx.x;
  uint32_t* w = reinterpret_cast<uint32_t*>(&s[0][0]);
  for (int i = lane; i < 8 * 64 * 4; i += 64) w[i] = 0xdead0000u + i;
  __syncthreads();
  uint32_t acc = lane;
  for (int it = 0; it < iters; ++it) {
    if (MODE & 1) acc = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((lane + it) & 63) << 2), (int)acc);
    if (MODE & 2) acc = (uint32_t)__builtin_amdgcn_ds_permute((int)(((lane * 5 + it) & 63) << 2), (int)acc);
    if (MODE & 4) {  // DMA into slots 4..7 while permuting
      __builtin_amdgcn_global_load_lds((gptr)(src + (it & 1023) * 64 + lane), (lptr)&s[4 + (it & 3)][0], 16, 0, 2);
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  uint32_t nb = 0;
  for (int i = lane; i < 4 * 64 * 4; i += 64) nb += w[i] != 0xdead0000u + i;  // slots 0..3 only
  // slots 4..7 hold the last DMA'd pieces: compare with the source
  if (MODE & 4) {
    for (int sl = 0; sl < 4; ++sl) {
      // the last piece written into slot (4 + sl) came from it = last index with (it & 3) == sl
      int last = iters - 1;
      while ((last & 3) != sl) --last;
      const uint4 want = src[(last & 1023) * 64 + lane];
      const uint4 got = s[4 + sl][lane];
      nb += (want.x != got.x) + (want.y != got.y) + (want.z != got.z) + (want.w != got.w);
    }
  }
  atomicAdd(bad, nb + (acc == 0x12345678u));
}

int main() {
  uint4* src;
  uint32_t* bad;
  const size_t n = 1024 * 64;
  (void)hipMalloc(&src, n * 16);
  (void)hipMalloc(&bad, 4);
  uint4* h = (uint4*)malloc(n * 16);
  for (size_t i = 0; i < n; ++i) h[i] = make_uint4(i, i * 3, i * 7, ~i);
  (void)hipMemcpy(src, h, n * 16, hipMemcpyHostToDevice);
  for (int mode : {1, 2, 3, 4, 5, 6, 7}) {
    (void)hipMemset(bad, 0, 4);
    if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(1024), dim3(64), 0, 0, src, bad, 4000);
    if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(1024), dim3(64), 0, 0, src, bad, 4000);
    if (mode == 3) hipLaunchKernelGGL(k<3>, dim3(1024), dim3(64), 0, 0, src, bad, 4000);
    if (mode == 4) hipLaunchKernelGGL(k<4>, dim3(1024), dim3(64), 0, 0, src, bad, 4000);
    if (mode == 5) hipLaunchKernelGGL(k<5>, dim3(1024), dim3(64), 0, 0, src, bad, 4000);
    if (mode == 6) hipLaunchKernelGGL(k<6>, dim3(1024), dim3(64), 0, 0, src, bad, 4000);
    if (mode == 7) hipLaunchKernelGGL(k<7>, dim3(1024), dim3(64), 0, 0, src, bad, 4000);
    uint32_t b = 0;
    (void)hipMemcpy(&b, bad, 4, hipMemcpyDeviceToHost);
    printf("{\"mode\":%d,\"bpermute\":%d,\"permute\":%d,\"dma\":%d,\"bad_words\":%u}\n", mode,
           mode & 1, (mode >> 1) & 1, (mode >> 2) & 1, b);
  }
  return 0;
}
