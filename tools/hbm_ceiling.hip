// SPDX-License-Identifier: BSD-2-Clause
// Measures the practical HBM read ceiling of this MI355X for the access
// shapes the RX kernels can use, so roofline fractions can be read against
// both the 8 TB/s spec and what a pure stream reaches:
//   reg   16-B loads to VGPRs (nontemporal or default policy), 8 in flight
//   lds   16-B LDS-DMA (global_load_lds_dwordx4), nt or default, 8 in flight
// Build: make tools/hbm_ceiling
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void read_reg(const u32x4* __restrict__ p, size_t n16,
                                                uint32_t* out) {
  uint32_t acc = 0;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 7 * stride < n16; i += 8 * stride) {
    u32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      v[u] = NT ? __builtin_nontemporal_load(p + i + u * stride) : p[i + u * stride];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  for (; i < n16; i += stride) {
    u32x4 v = p[i];
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;  // keep the loads alive
}

// Each wave streams 1-KiB pieces into an 8-slot LDS ring by LDS-DMA and
// consumes each piece with one ds_read_b128 per lane.
template <int AUX>
__global__ __launch_bounds__(256) void read_lds(const u32x4* __restrict__ p, size_t n16,
                                                uint32_t* out) {
  __shared__ __attribute__((aligned(16))) u32x4 ring[4][8][64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t waves = (size_t)gridDim.x * 4;
  const size_t gw = (size_t)blockIdx.x * 4 + w;
  const size_t npieces = n16 / 64;
  uint32_t acc = 0;
  for (size_t b = gw * 8; b < npieces; b += waves * 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const size_t piece = b + u;
      if (piece < npieces)
        __builtin_amdgcn_global_load_lds((const void*)(p + piece * 64 + lane), (void __attribute__((address_space(3)))*)&ring[w][u][0], 16, 0, AUX);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const u32x4 v = ring[w][u][lane];
      acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <typename K>
static float time_it(K kern, int grid, const u32x4* a, size_t n16, uint32_t* o) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e9f;
  for (int r = 0; r < 12; ++r) {
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, a, n16, o);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (r >= 2 && ms < best) best = ms;
  }
  return best;
}

// "ramp" mode (argv[2]): the stream ceiling launch by launch from a cold
// start, the way bench.py's driver window sees it -- after an idle second,
// `launches` back-to-back launches of the LDS-DMA stream (nt, 8 waves per
// CU), each timed by its own event pair; prints the per-launch GB/s and the
// means over launches 6-25 (bench.py's --warmup 5 --steps 20 window) and
// 26-225 (its `steady` side measurement).
static int ramp(const u32x4* a, size_t bytes, uint32_t* o, int cu, int launches) {
  const size_t n16 = bytes / 16;
  hipEvent_t* e = (hipEvent_t*)malloc(sizeof(hipEvent_t) * (launches + 1));
  for (int i = 0; i <= launches; ++i) (void)hipEventCreate(&e[i]);
  (void)hipDeviceSynchronize();
  const hipError_t s = hipDeviceSynchronize();
  if (s != hipSuccess) return 1;
  // (idle: the clocks drop as they do between bench.py's setup and its warm-up)
  struct timespec ts = {1, 0};
  nanosleep(&ts, nullptr);
  (void)hipEventRecord(e[0], 0);
  for (int i = 0; i < launches; ++i) {
    hipLaunchKernelGGL(read_lds<2>, dim3(cu * 8), dim3(256), 0, 0, a, n16, o);
    (void)hipEventRecord(e[i + 1], 0);
  }
  (void)hipEventSynchronize(e[launches]);
  double w = 0, sdy = 0;
  int nw = 0, ns = 0;
  printf("{\"bytes\":%zu,\"gbps\":[", bytes);
  for (int i = 0; i < launches; ++i) {
    float ms;
    (void)hipEventElapsedTime(&ms, e[i], e[i + 1]);
    const double g = bytes / (ms * 1e-3) / 1e9;
    printf("%s%.1f", i ? "," : "", g);
    if (i >= 5 && i < 25) { w += ms; ++nw; }
    if (i >= 25) { sdy += ms; ++ns; }
  }
  printf("],\"window_6_25_GBps\":%.1f,\"steady_26_GBps\":%.1f}\n",
         nw ? bytes / (w / nw * 1e-3) / 1e9 : 0.0, ns ? bytes / (sdy / ns * 1e-3) / 1e9 : 0.0);
  return 0;
}

int main(int argc, char** argv) {
  const size_t bytes = (argc > 1 ? strtoull(argv[1], 0, 0) : (size_t)2 << 30);
  const size_t n16 = bytes / 16;
  u32x4* a;
  uint32_t* o;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&o, 4) != hipSuccess) return 1;
  (void)hipMemset(a, 1, bytes);
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int cu = prop.multiProcessorCount;
  if (argc > 2 && argv[2][0] == 'r') return ramp(a, bytes, o, cu, argc > 3 ? atoi(argv[3]) : 225);
  for (int m : {4, 8, 16, 32}) {
    const int g = cu * m;
    const float t1 = time_it(read_reg<true>, g, a, n16, o);
    const float t2 = time_it(read_reg<false>, g, a, n16, o);
    const float t3 = time_it(read_lds<2>, g, a, n16, o);
    const float t4 = time_it(read_lds<0>, g, a, n16, o);
    printf("{\"grid\":%d,\"bytes\":%zu,\"reg_nt_GBps\":%.1f,\"reg_GBps\":%.1f,"
           "\"lds_nt_GBps\":%.1f,\"lds_GBps\":%.1f}\n",
           g, bytes, bytes / (t1 * 1e-3) / 1e9, bytes / (t2 * 1e-3) / 1e9,
           bytes / (t3 * 1e-3) / 1e9, bytes / (t4 * 1e-3) / 1e9);
  }
  return 0;
}
