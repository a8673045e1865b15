// SPDX-License-Identifier: BSD-2-Clause
// Streaming-ring probe: how much LDS-DMA must a CU keep in flight to read
// HBM near its ceiling when every wave streams through a continuous ring of
// R 1-KiB slots with a counted `s_waitcnt vmcnt(R-1)` (never a full drain)?
// Each wave owns a contiguous span of the buffer.  Prints one JSON line per
// (slots per wave, waves per block, blocks per CU).
// Build: make tools/ring_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short v2u16 __attribute__((ext_vector_type(2)));

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ uint32_t dot(uint32_t w, uint32_t acc) {
  return __builtin_amdgcn_udot2(__builtin_bit_cast(v2u16, w),
                                __builtin_bit_cast(v2u16, 0x00010001u), acc, false);
}

template <int R, int W>
__global__ __launch_bounds__(64 * W) void ring(const u32x4* __restrict__ p, size_t npieces,
                                               uint32_t* out) {
  extern __shared__ __attribute__((aligned(16))) u32x4 lds[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  u32x4* slot0 = lds + (size_t)w * R * 64;
  const size_t waves = (size_t)gridDim.x * W;
  const size_t gw = (size_t)blockIdx.x * W + w;
  const size_t per = (npieces + waves - 1) / waves;
  const size_t b = gw * per;
  const size_t e = b + per < npieces ? b + per : npieces;
  uint32_t acc = 0;
  if (b < e) {
    const size_t last = e - 1;
    // prologue: R pieces in flight (pieces past the span reload the last one)
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const size_t pc = b + u <= last ? b + u : last;
      __builtin_amdgcn_global_load_lds((const void*)(p + pc * 64 + lane),
                                       (void __attribute__((address_space(3)))*)(slot0 + u * 64),
                                       16, 0, 2);
    }
    for (size_t i = b; i < e; i += R) {
#pragma unroll
      for (int u = 0; u < R; ++u) {
        wait_vm<R - 1>();
        const u32x4 v = slot0[u * 64 + lane];
        acc = dot(v.x, dot(v.y, dot(v.z, dot(v.w, acc))));
        const size_t nx = i + R + u;
        const size_t pc = nx <= last ? nx : last;
        __builtin_amdgcn_global_load_lds((const void*)(p + pc * 64 + lane),
                                         (void __attribute__((address_space(3)))*)(slot0 + u * 64),
                                         16, 0, 2);
      }
    }
    wait_vm<0>();
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <int R, int W>
static void run(const u32x4* a, size_t bytes, uint32_t* o, int cu) {
  const size_t lds = (size_t)R * W * 1024;
  int bpc = 0;
  (void)hipFuncSetAttribute((const void*)ring<R, W>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds);
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, ring<R, W>, 64 * W, lds);
  for (int m : {1, 2, 3, 4, 5, 6, 8, 10, 12, 16}) {
    if (m > bpc) break;
    const int grid = cu * m;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e9f;
    for (int r = 0; r < 10; ++r) {
      (void)hipEventRecord(e0, 0);
      hipLaunchKernelGGL((ring<R, W>), dim3(grid), dim3(64 * W), lds, 0, a, bytes / 1024, o);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (r >= 2 && ms < best) best = ms;
    }
    printf("{\"slots\":%d,\"waves_per_block\":%d,\"blocks_per_cu\":%d,\"kib_in_flight_per_cu\":%d,"
           "\"GBps\":%.1f}\n",
           R, W, m, R * W * m, bytes / (best * 1e-3) / 1e9);
  }
}


// Grouped variant: each wave owns 64-frame tiles of FB-byte frames; groups
// of G lanes stream one frame each (G*16 contiguous bytes per round), so an
// instruction touches 64/G frames.
template <int R, int G, int FB = 1536, bool AL = false>
__global__ __launch_bounds__(64) void ring_grp(const u32x4* __restrict__ p, size_t nframes,
                                               uint32_t* out) {
  // frames of FB bytes at FB-byte stride (16-B aligned starts: FB 1536, or
  // not: 1514, whose 16-B chunk runs straddle 128-B lines)
  // AL: rounds start on the 128-B line at or below the frame (one more
  // chunk run per frame; the extra bytes would be masked)
  constexpr uint32_t fb16 = (FB + 15) / 16 + (AL ? 8 : 0);
  extern __shared__ __attribute__((aligned(16))) u32x4 lds[];
  const int lane = threadIdx.x;
  const int g = lane / G, j = lane % G;
  constexpr int NG = 64 / G;
  const size_t ntiles = nframes / 64;
  constexpr uint32_t rounds = (fb16 + G - 1) / G;  // rounds per frame per group
  uint32_t acc = 0;
  for (size_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    // group g streams frames t*64 + g, + NG, ...: (64/NG) frames x rounds
    const uint32_t total = (64 / NG) * rounds;
    auto src = [&](uint32_t k) {
      const uint32_t fi = k / rounds, r = k % rounds;
      const uint32_t c = r * G + j;
      const size_t frame = t * 64 + g + fi * NG;
      const size_t b16 = AL ? ((frame * FB) & ~(size_t)127) / 16 : (frame * FB) / 16;
      return (k < total && c < fb16) ? p + b16 + c : p;
    };
#pragma unroll
    for (int u = 0; u < R; ++u)
      __builtin_amdgcn_global_load_lds((const void*)src(u), (void __attribute__((address_space(3)))*)(lds + u * 64), 16, 0, 2);
    for (uint32_t k0 = 0; k0 < total; k0 += R) {
#pragma unroll
      for (int u = 0; u < R; ++u) {
        wait_vm<R - 1>();
        const u32x4 v = lds[u * 64 + lane];
        acc = dot(v.x, dot(v.y, dot(v.z, dot(v.w, acc))));
        __builtin_amdgcn_global_load_lds((const void*)src(k0 + R + u), (void __attribute__((address_space(3)))*)(lds + u * 64), 16, 0, 2);
      }
    }
    wait_vm<0>();
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// Split variant: each tile first reads line 0 of its 64 frames (8
// instructions of eight frames x 128 B, as rx_kernel stages header windows),
// then the other FB/128 - 1 lines of each frame by 8-lane groups.  HDRLAG:
// the line-0 reads are for the NEXT tile (as rx_kernel's pipelined staging).
template <int R, bool HDRLAG, int ST = 0, int HAUX = 0, int SEC = 0, int BAUX = 2>
__global__ __launch_bounds__(64) void ring_split(const u32x4* __restrict__ p, size_t nframes,
                                                 uint32_t* out) {
  constexpr uint32_t fb16 = 96, lines = 12;
  extern __shared__ __attribute__((aligned(16))) u32x4 lds[];
  const int lane = threadIdx.x;
  const int g = lane / 8, j = lane % 8;
  const size_t ntiles = nframes / 64;
  uint32_t acc = 0;
  uint32_t pend = 0;  // ST 11: tiles whose records wait for the next write window
  for (size_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const size_t th = HDRLAG ? t + gridDim.x : t;
    if (th < ntiles) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const size_t frame = th * 64 + i * 8 + g;
        __builtin_amdgcn_global_load_lds((const void*)(p + frame * fb16 + j),
                                         (void __attribute__((address_space(3)))*)(lds + (R + i) * 64),
                                         16, 0, HAUX);
      }
    }
    const uint32_t total = 8 * (lines - 1);  // rounds: 8 frames per group x 11 lines
    auto src = [&](uint32_t k) {
      const uint32_t fi = k / (lines - 1), r = k % (lines - 1) + 1;
      const size_t frame = t * 64 + g + fi * 8;
      return k < total ? p + frame * fb16 + r * 8 + j : p;
    };
    // SEC: lanes 4-7 of each group read their line's lower half again, so
    // only the lower 64 B of every body line is requested
    auto srcs = [&](uint32_t k) {
      return (SEC != 0 && k < total && j >= 4) ? src(k) - 4 : src(k);
    };
#pragma unroll
    for (int u = 0; u < R; ++u)
      __builtin_amdgcn_global_load_lds((const void*)srcs(u), (void __attribute__((address_space(3)))*)(lds + u * 64), 16, 0, BAUX);
    for (uint32_t k0 = 0; k0 < total; k0 += R) {
#pragma unroll
      for (int u = 0; u < R; ++u) {
        wait_vm<R - 1>();
        const u32x4 v = lds[u * 64 + lane];
        acc = dot(v.x, dot(v.y, dot(v.z, dot(v.w, acc))));
        __builtin_amdgcn_global_load_lds((const void*)srcs(k0 + R + u), (void __attribute__((address_space(3)))*)(lds + u * 64), 16, 0, BAUX);
      }
    }
    wait_vm<0>();
    const u32x4 h = lds[R * 64 + lane];
    acc += h.x;
    if (ST) {  // a 32-B record per frame, like rx_kernel's (1: default policy, 2: nontemporal)
      u32x4* rec = reinterpret_cast<u32x4*>(out) + 16 + (t * 64 + lane) * 2;
      const u32x4 r0 = {acc, acc + 1, acc + 2, acc + 3};
      if (ST == 1) {
        rec[0] = r0;
        rec[1] = r0;
      } else if (ST == 2) {
        __builtin_nontemporal_store(r0, rec);
        __builtin_nontemporal_store(r0, rec + 1);
      } else if (ST == 3) {
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\tglobal_store_dwordx4 %0, %1, off offset:16 sc1"
                     ::"v"(rec), "v"(r0) : "memory");
      } else if (ST == 4) {
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\tglobal_store_dwordx4 %0, %1, off offset:16 sc0 sc1"
                     ::"v"(rec), "v"(r0) : "memory");
      } else if (ST == 5) {
        asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\tglobal_store_dwordx4 %0, %1, off offset:16 nt sc1"
                     ::"v"(rec), "v"(r0) : "memory");
      } else if (ST == 7) {  // two lanes per record: each instruction writes 1 KiB of whole lines
        u32x4* rq = reinterpret_cast<u32x4*>(out) + 16 + t * 128 + lane;
        rq[0] = r0;
        rq[64] = r0;
      } else if (ST == 8 || ST == 9 || ST == 10) {  // 8 / 2 tiles' records at once; 4 with nt stores
        constexpr int K = ST == 8 ? 8 : ST == 9 ? 2 : 4;
        if ((t / gridDim.x) % K == K - 1) {
          for (int q = 0; q < K; ++q) {
            u32x4* rq = reinterpret_cast<u32x4*>(out) + 16 + ((t - q * gridDim.x) * 64 + lane) * 2;
            if (ST == 10) {
              __builtin_nontemporal_store(r0, rq);
              __builtin_nontemporal_store(r0, rq + 1);
            } else {
              rq[0] = r0;
              rq[1] = r0;
            }
          }
        }
      } else if (ST == 11) {  // all waves write in the same 1.28-us window of every 10.24 us
        ++pend;
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (((now >> 7) & 7u) == 0 || pend >= 8 || t + gridDim.x >= ntiles) {
          for (uint32_t q = 0; q < pend; ++q) {
            u32x4* rq = reinterpret_cast<u32x4*>(out) + 16 + ((t - q * gridDim.x) * 64 + lane) * 2;
            rq[0] = r0;
            rq[1] = r0;
          }
          pend = 0;
        }
      } else if ((t / gridDim.x) % 4 == 3) {  // 6: four tiles' records at once (8 KB)
        for (int q = 0; q < 4; ++q) {
          u32x4* rq = reinterpret_cast<u32x4*>(out) + 16 + ((t - q * gridDim.x) * 64 + lane) * 2;
          rq[0] = r0;
          rq[1] = r0;
        }
      }
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <int R, bool HDRLAG, int ST = 0, int HAUX = 0, int SEC = 0, int BAUX = 2>
static void run_split(const u32x4* a, size_t bytes, uint32_t* o, int cu, const char* tag = "") {
  const size_t lds = (size_t)(R + 8) * 1024;
  const size_t nframes = (bytes - 4096) / 1536 / 64 * 64;
  for (int m : {8, 10}) {
    const int grid = cu * m;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e9f;
    for (int r = 0; r < 10; ++r) {
      (void)hipEventRecord(e0, 0);
      hipLaunchKernelGGL((ring_split<R, HDRLAG, ST, HAUX, SEC, BAUX>), dim3(grid), dim3(64), lds, 0, a, nframes, o);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (r >= 2 && ms < best) best = ms;
    }
    printf("{\"split_hdr\":1,\"tag\":\"%s\",\"hdr_aux\":%d,\"body_aux\":%d,\"half_lines\":%d,\"hdr_lag\":%d,\"stores\":%d,\"slots\":%d,\"waves_per_cu\":%d,\"ms\":%.4f,\"GBps\":%.1f}\n",
           tag, HAUX, BAUX, SEC, (int)HDRLAG, ST, R, m, best, nframes * 1536 / (best * 1e-3) / 1e9);
  }
}

template <int R, int G, int FB = 1536, bool AL = false>
static void run_grp(const u32x4* a, size_t bytes, uint32_t* o, int cu) {
  const size_t lds = (size_t)R * 1024;
  const size_t nframes = (bytes - 4096) / FB / 64 * 64;
  int bpc = 0;
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, ring_grp<R, G, FB, AL>, 64, lds);
  for (int m : {4, 8, 10, 12, 16}) {
    if (m > bpc) break;
    const int grid = cu * m;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e9f;
    for (int r = 0; r < 10; ++r) {
      (void)hipEventRecord(e0, 0);
      hipLaunchKernelGGL((ring_grp<R, G, FB, AL>), dim3(grid), dim3(64), lds, 0, a, nframes, o);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (r >= 2 && ms < best) best = ms;
    }
    if (hipGetLastError() != hipSuccess) { printf("launch error\n"); exit(1); }
    printf("{\"grouped\":%d,\"aligned_rounds\":%d,\"frame\":%d,\"slots\":%d,\"waves_per_cu\":%d,\"GBps\":%.1f}\n", G, (int)AL, FB,
           (int)AL, R, m, nframes * FB / (best * 1e-3) / 1e9);
  }
}

int main(int argc, char** argv) {
  const size_t bytes = (argc > 1 ? strtoull(argv[1], 0, 0) : (size_t)1610612736);
  u32x4* a;
  uint32_t* o;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&o, bytes / 40 + 4096) != hipSuccess) return 1;
  (void)hipMemset(a, 1, bytes);
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int cu = prop.multiProcessorCount;
  if (argc > 2 && argv[2][0] == 'r') {
    run<8, 1>(a, bytes, o, cu);
    run<16, 1>(a, bytes, o, cu);
    run<32, 1>(a, bytes, o, cu);
  }
  if (argc > 2 && argv[2][0] == 'w') {  // write cost by write grouping (round 3)
    for (int rep = 0; rep < 3; ++rep) {
      run_split<4, true, 0>(a, bytes, o, cu, "reads");
      run_split<4, true, 1>(a, bytes, o, cu, "records");
      run_split<4, true, 9>(a, bytes, o, cu, "records_2tiles");
      run_split<4, true, 6>(a, bytes, o, cu, "records_4tiles");
      run_split<4, true, 8>(a, bytes, o, cu, "records_8tiles");
      run_split<4, true, 10>(a, bytes, o, cu, "records_4tiles_nt");
      run_split<4, true, 2>(a, bytes, o, cu, "records_nt");
      run_split<4, true, 11>(a, bytes, o, cu, "records_time_window");
    }
    return 0;
  }
  if (argc > 2 && argv[2][0] == 'c') {  // 60 back-to-back launches (per-launch clock under rocprofv3)
    const size_t nframes = (bytes - 4096) / 1536 / 64 * 64;
    const int grid = cu * 10;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < 60; ++r)
      hipLaunchKernelGGL((ring_split<4, true, 1>), dim3(grid), dim3(64), (size_t)(4 + 8) * 1024, 0, a,
                         nframes, o);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("{\"tag\":\"records_60_launches\",\"ms_per_launch\":%.4f}\n", ms / 60);
    return 0;
  }
  if (argc > 2 && argv[2][0] == 'h') {  // one variant per run, for rocprofv3 --pmc
    if (argv[2][1] == '1') run_split<4, true, 0, 0, 1>(a, bytes, o, cu, "reads_half_body_lines");
    else run_split<4, true, 0>(a, bytes, o, cu, "reads");
    return 0;
  }
  run_split<4, true>(a, bytes, o, cu);
  run_split<4, true, 1>(a, bytes, o, cu);
  run_split<4, true, 2>(a, bytes, o, cu);
  run_split<4, true, 3>(a, bytes, o, cu);
  run_split<4, true, 4>(a, bytes, o, cu);
  run_split<4, true, 5>(a, bytes, o, cu);
  run_split<4, true, 6>(a, bytes, o, cu);
  return 0;
}
