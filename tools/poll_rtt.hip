// SPDX-License-Identifier: BSD-2-Clause
//
// poll_rtt -- the fixed costs under a device poll of a few events (DESIGN.md
// §5e, VERDICT r4 "missing #2"): how long the host waits, per poll, before a
// single frame's verdict can be back, for
//   launch_sync    an empty kernel launched and waited for (hipStreamSynchronize):
//                  what the per-poll launch + completion wait of the shim costs;
//   launch_flag    the same launch, completion seen by spinning on a host word
//                  the kernel stores (no HIP wait call);
//   resident_ping  a resident kernel spinning on a host doorbell, answering in
//                  a host word: the floor of any device path (one PCIe round
//                  trip each way, no launch);
//   resident_read  the same, the kernel first reading 64 x 128 B of frame
//                  windows from host memory (one more PCIe round trip: the
//                  least a verdict needs).
// The resident kernel leaves its loop after `iters` pings or two seconds of
// wall time, whichever comes first, so the grid always drains.
//
//   tools/poll_rtt [iters]   -> one JSON line per mode (median / p10 / p90 us)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

namespace {

constexpr uint64_t kDeadlineTicks = 200000000ull;  // 2 s of s_memrealtime (100 MHz)

__device__ __forceinline__ uint32_t sys_load(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void sys_store(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void empty_kernel(uint32_t* flag, uint32_t v) {
  if (flag != nullptr && threadIdx.x == 0) sys_store(flag, v);
}

// One wave.  Ping i: wait for doorbell == i, optionally read the window
// rows, then ack = i (+ a data-dependent term so the reads are not dropped).
__global__ void resident(const uint32_t* doorbell, uint32_t* ack, const uint4* frames, uint32_t iters,
                         uint32_t* sink) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t acc = 0;
  for (uint32_t i = 1; i <= iters; ++i) {
    bool late = false;
    for (;;) {
      if (sys_load(doorbell) >= i) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > kDeadlineTicks) {
        late = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (late) break;
    if (frames != nullptr) {
      // 64 frames x 128 B: lane l reads frame l's eight 16-B cells
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      const u32x4* f = reinterpret_cast<const u32x4*>(frames) + (size_t)threadIdx.x * 8;
      u32x4 v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = __builtin_nontemporal_load(f + k);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc += v[k].x ^ v[k].w;
    }
    if (threadIdx.x == 0) sys_store(ack, i);
  }
  if (acc == 0xdeadbeefu) sink[threadIdx.x] = acc;
}

struct Stats {
  double med, p10, p90;
};
Stats stats(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  auto q = [&](double f) { return v[std::min(v.size() - 1, (size_t)(f * (double)v.size()))]; };
  return {q(0.5), q(0.1), q(0.9)};
}

void report(const char* mode, const std::vector<double>& us) {
  const Stats s = stats(us);
  printf("{\"mode\": \"%s\", \"n\": %zu, \"us_median\": %.2f, \"us_p10\": %.2f, \"us_p90\": %.2f}\n", mode,
         us.size(), s.med, s.p10, s.p90);
  fflush(stdout);
}

double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// Host spin with its own two-second deadline; false on timeout.
bool spin_until(volatile uint32_t* p, uint32_t v) {
  const double t0 = now_us();
  while (__atomic_load_n(p, __ATOMIC_ACQUIRE) < v)
    if (now_us() - t0 > 2e6) return false;
  return true;
}

}  // namespace

int main(int argc, char** argv) {
  const uint32_t iters = argc > 1 ? (uint32_t)atoi(argv[1]) : 2000;
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  uint32_t* words;  // [0] doorbell, [32] ack, [64] launch flag (separate lines)
  CHECK(hipHostMalloc(&words, 4096, hipHostMallocCoherent | hipHostMallocMapped));
  for (int i = 0; i < 1024; ++i) words[i] = 0;
  uint32_t *d_words, *sink;
  CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&d_words), words, 0));
  CHECK(hipMalloc(&sink, 256));
  uint8_t* frames;
  CHECK(hipHostMalloc(&frames, 64 * 128, hipHostMallocDefault));
  for (int i = 0; i < 64 * 128; ++i) frames[i] = (uint8_t)i;
  uint4* d_frames;
  CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&d_frames), frames, 0));

  // warm the runtime
  hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, nullptr, 0u);
  CHECK(hipStreamSynchronize(s));

  std::vector<double> us;
  for (uint32_t i = 0; i < iters; ++i) {
    const double t = now_us();
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, nullptr, 0u);
    CHECK(hipStreamSynchronize(s));
    us.push_back(now_us() - t);
  }
  report("launch_sync", us);

  us.clear();
  volatile uint32_t* flag = words + 64;
  for (uint32_t i = 1; i <= iters; ++i) {
    const double t = now_us();
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, d_words + 64, i);
    if (!spin_until(flag, i)) {
      fprintf(stderr, "launch_flag: timeout\n");
      break;
    }
    us.push_back(now_us() - t);
  }
  CHECK(hipStreamSynchronize(s));
  report("launch_flag", us);

  for (int mode = 0; mode < 2; ++mode) {
    volatile uint32_t* doorbell = words;
    volatile uint32_t* ack = words + 32;
    *doorbell = 0;
    *ack = 0;
    hipLaunchKernelGGL(resident, dim3(1), dim3(64), 0, s, d_words, d_words + 32,
                       mode ? d_frames : nullptr, iters, sink);
    us.clear();
    for (uint32_t i = 1; i <= iters; ++i) {
      const double t = now_us();
      __atomic_store_n(doorbell, i, __ATOMIC_RELEASE);
      if (!spin_until(ack, i)) {
        fprintf(stderr, "resident: timeout at %u\n", i);
        break;
      }
      us.push_back(now_us() - t);
    }
    // the kernel ends after its last ping (or its own deadline)
    CHECK(hipStreamSynchronize(s));
    report(mode ? "resident_read" : "resident_ping", us);
  }
  CHECK(hipHostFree(words));
  CHECK(hipHostFree(frames));
  CHECK(hipFree(sink));
  CHECK(hipStreamDestroy(s));
  return 0;
}
