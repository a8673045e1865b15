// SPDX-License-Identifier: BSD-2-Clause
//
// oo_rx_kernel.hip -- gfx950 (MI355X / CDNA4) kernels for Onload's software
// receive transform: checksum verify + header parse + 4-tuple socket demux.
//
// Reference semantics (file:line in /root/reference):
//   handle_rx_csum_bad            src/lib/transport/ip/netif_event.c:1014-1128
//   ci_parse_rx_vlan              netif_event.c:116-132
//   ci_ip_csum_correct            netif_event.c:80-94 (+ citools/ip_csum_partial.c:20-39)
//   ci_tcp_csum_correct           netif_event.c:97-113
//   ci_udp_csum_correct           src/lib/transport/ip/udp_rx.c:101-121
//   ef_{udp,tcp}_checksum*_is_correct  src/lib/ciul/checksum.c:298-351
//   handle_rx_pkt                 netif_event.c:250-451
//   ci_ip_options_parse           netif_event.c:135-185
//   ci_udp_handle_rx              udp_rx.c:236-307
//   ci_tcp_handle_rx              src/lib/transport/ip/tcp_rx.c:4681-4836
//   ci_netif_filter_for_each_match[_ip6]  netif_table.c:234-319, netif_table_ip6.c:110-189
//   __onload_hash1/2/3            src/include/onload/hash.h:84-173
//
// Work unit: a tile of up to 64 packets.  Per packet the transform splits
// into
//   * the header work: the first 128 bytes of the frame (the "window") are
//     parsed one packet per lane -- VLAN, L3/L4 gates, pseudo-header, IPv4
//     header sum, the L4 sum inside the window, handle_rx_pkt's
//     frag/options/TCP-scattered tests and the 2 or 3 lookup stages --
//     giving a 32-B record that is final unless the L4 region runs past the
//     window (parse_headers, demux_packet);
//   * the body: the frame bytes past the window, summed by 8-lane groups
//     (128 contiguous bytes per group per round, one packet per group at a
//     time) from a ring of 1-KiB LDS-DMA pieces (Body).  Only the
//     descriptors decide the body, so it can be in flight before the parse.
// The verdict of a long packet adds the body sum to the window part.
//
// One kernel, rx_kernel: every wave parses and streams its own tiles
// (DESIGN.md §2); tx_kernel runs the same tile loop for the TX fill.
// Every frame-byte and descriptor read in the streaming code is an LDS-DMA
// (global_load_lds_dwordx4) whose completion the wave counts itself with
// s_waitcnt vmcnt(N); the LDS reads that follow are inline asm, because
// hipcc waits vmcnt(0) before any LDS access it sees while LDS-DMA is in
// flight.
//
// The verdict uses the mod-0xffff residue of the exact word sum; see
// oracle/rx_oracle.c for why that equals the reference's folded-complement
// test (and why it may be summed in any grouping).  No MFMA: integer
// reduction + table probes, HBM-bound.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "oo_rx_device.h"

// OO_RX_SHORT (oo_rx_kernel_short.hip): the same rx_kernel with a 2-slot
// ring, compiled into namespace oo_rx_short for short-frame batches (no
// tx_kernel there: its check-field staging needs a 4-slot ring).
// OO_RX_POLL (oo_rx_kernel_poll.hip): rx_kernel alone, for a poll's batch,
// in namespace oo_rx_poll (see "The poll instance" at its kernel).
#if defined(OO_RX_POLL)
namespace oo_rx_poll {
using namespace ::oo_rx;
#elif defined(OO_RX_SHORT)
namespace oo_rx_short {
using namespace ::oo_rx;
#else
namespace oo_rx {
#endif

typedef unsigned short v2u16 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Tuning knobs (compile-time; `make variants` builds sweeps of them).
#ifndef OO_RX_WAVES
#define OO_RX_WAVES 2  // rx_kernel: waves per block
#endif
#ifndef OO_RX_RING
#define OO_RX_RING 4  // rx_kernel: body ring slots per wave (even)
#endif
#ifndef OO_RX_GSEQ
#define OO_RX_GSEQ 0  // 1: per-group job sequences instead of lockstep job slots
#endif

constexpr int WAVES = OO_RX_WAVES;
constexpr int R = OO_RX_RING;
static_assert(R % 2 == 0, "rx_kernel consumes its ring two pieces at a time");
constexpr int HC = 8;                // staged header chunks per packet
constexpr int HB = HC * 16;          // staged window bytes per packet
static_assert(HB == (int)HB_BYTES, "oo_rx_device.h HB_BYTES");

constexpr uint32_t PENDING = 0xffu;

typedef const __attribute__((address_space(1))) void* gptr;
typedef __attribute__((address_space(3))) void* lptr;

// One 16-byte LDS-DMA per lane (global_load_lds_dwordx4, nontemporal): lane
// l's bytes land at lds + 16 l (lds is wave-uniform).  The global address is
// forced to the global address space: a pointer rebuilt from integers would
// otherwise be a flat access.
template <int AUX = 2>
__device__ __forceinline__ void glds(uint64_t src, void* lds) {
  __builtin_amdgcn_global_load_lds(reinterpret_cast<gptr>(src), (lptr)(lds), 16, 0, AUX);
}
#ifndef OO_RX_HDR_AUX
#define OO_RX_HDR_AUX 0  // header window: default policy (its lines are hit 8 times)
#endif
#ifndef OO_RX_BODY_AUX
#define OO_RX_BODY_AUX 2  // body stream: nontemporal
#endif

// Wait until at most N of this wave's vector-memory operations (loads,
// LDS-DMA and stores, which retire in issue order) are outstanding.
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// LDS reads the compiler cannot see.  While LDS-DMA is in flight hipcc waits
// vmcnt(0) before any LDS access it cannot prove disjoint from the DMA
// target, which would drain the ring on every read; these reads carry their
// own lgkmcnt wait, and their ordering after the DMA is the caller's counted
// vm_wait.
__device__ __forceinline__ uint4 lds_read16(const void* p) {
  uint4 v;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)"
               : "=v"(v)
               : "v"((uint32_t)(uintptr_t)(lptr)(p))
               : "memory");
  return v;
}

// Two 16-B LDS reads, one wait (early-clobber outputs: the second read must
// not take its address from a register the first is already writing).
__device__ __forceinline__ void lds_read16x2(const void* p0, const void* p1, uint4& v0, uint4& v1) {
  asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %3\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(v0), "=&v"(v1)
               : "v"((uint32_t)(uintptr_t)(lptr)(p0)), "v"((uint32_t)(uintptr_t)(lptr)(p1))
               : "memory");
}

// Value of v in lane src (ds_bpermute: no LDS memory access, so it needs no
// vmcnt wait).  Call with every lane active.
__device__ __forceinline__ uint32_t lane_get(uint32_t v, uint32_t src) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v);
}

__device__ __forceinline__ uint32_t fold16(uint32_t s) {
  s = (s & 0xffffu) + (s >> 16);
  s = (s & 0xffffu) + (s >> 16);
  return s;
}
__device__ __forceinline__ uint32_t swap16(uint32_t f) {
  return ((f & 0xffu) << 8) | (f >> 8);
}

__device__ __forceinline__ uint32_t dot(uint32_t w, uint32_t m, uint32_t acc) {
  return __builtin_amdgcn_udot2(__builtin_bit_cast(v2u16, w), __builtin_bit_cast(v2u16, m),
                                acc, false);
}

// Sum of all eight LE u16 words of a chunk.
__device__ __forceinline__ uint32_t chunk_sum_all(const uint4& v, uint32_t acc) {
  acc = dot(v.x, 0x00010001u, acc);
  acc = dot(v.y, 0x00010001u, acc);
  acc = dot(v.z, 0x00010001u, acc);
  return dot(v.w, 0x00010001u, acc);
}

// Sum of the LE u16 words of one 16-byte chunk at window position p,
// restricted to window bytes [S, E).  Words pair at even window positions;
// an odd S or E clips half a word, removed by subtracting that byte (the low
// byte of the word at S-1, or the high byte of the word at E-1).
__device__ __forceinline__ uint32_t chunk_sum(const uint4& v, int p, int S, int E) {
  int lo = (S & ~1) - p;
  int hi = ((E + 1) & ~1) - p;
  lo = lo < 0 ? 0 : lo;
  hi = hi > 16 ? 16 : hi;
  uint32_t wm = 0;
  if (hi > lo) wm = ((1u << (hi >> 1)) - 1u) & ~((1u << (lo >> 1)) - 1u);
  uint32_t s = 0;
  s = dot(v.x, (wm & 1u) | ((wm & 2u) << 15), s);
  s = dot(v.y, ((wm >> 2) & 1u) | ((wm & 8u) << 13), s);
  s = dot(v.z, ((wm >> 4) & 1u) | ((wm & 32u) << 11), s);
  s = dot(v.w, ((wm >> 6) & 1u) | ((wm & 128u) << 9), s);
  if (((S | E) & 1) != 0) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    if ((S & 1) && S - 1 >= p && S - 1 < p + 16) {
      const int b = S - 1 - p;
      s -= (w[b >> 2] >> ((b & 3) * 8)) & 0xffu;
    }
    if ((E & 1) && E >= p && E < p + 16) {
      const int b = E - p;
      s -= ((w[b >> 2] >> ((b & 3) * 8)) & 0xffu) << 8;
    }
  }
  return s;
}

#if (defined(OO_RX_STAMPS) || defined(OO_RX_PAD_VALU) || defined(OO_RX_BOUND_NOLOOK) || defined(OO_RX_BOUND_NOBODY) || \
     defined(OO_RX_BOUND_KXLINE) || defined(OO_RX_BOUND_KX1) || defined(OO_RX_BOUND_NOGENSUM)) && \
    !defined(OO_RX_EXPERIMENTS)
#error "OO_RX_STAMPS is a diagnostic build (tools/build_ref.sh sets OO_RX_EXPERIMENTS)"
#endif
#ifdef OO_RX_STAMPS
// Diagnostic phase stamps: stamps[((wave * 128 + iter) * 16) + phase] = realtime
// (100 MHz) for the first 128 tiles of each wave.
#define STAMP(ph, val)                                                                \
  do {                                                                                \
    if (P.stamps != nullptr && lane == 0 && it_ < 128)                               \
      P.stamps[((size_t)gwave * 128 + it_) * 16 + (ph)] = (val);                      \
  } while (0)
// Inside the demux (phases 8..10): the tile loop points dstamp at its slots.
__device__ uint64_t* dstamp_slot(uint64_t* p = nullptr, bool set = false) {
  static __shared__ uint64_t* slot[4];
  const uint32_t w = threadIdx.x >> 6;
  if (set) slot[w] = p;
  return slot[w];
}
#define DSTAMP(ph)                                                                    \
  do {                                                                                \
    uint64_t* dp_ = dstamp_slot();                                                    \
    if (dp_ != nullptr && __builtin_amdgcn_mbcnt_lo(~0u, 0u) == 0)                    \
      dp_[(ph)] = __builtin_amdgcn_s_memrealtime();                                   \
  } while (0)
#define DSTAMPV(ph, v)                                                                \
  do {                                                                                \
    uint64_t* dp_ = dstamp_slot();                                                    \
    if (dp_ != nullptr && __builtin_amdgcn_mbcnt_lo(~0u, 0u) == 0) dp_[(ph)] = (v);   \
  } while (0)
#define DSTAMPA(ph)                                                                   \
  do {                                                                                \
    uint64_t* dp_ = dstamp_slot();                                                    \
    const uint64_t ex_ = __ballot(1);                                                 \
    if (dp_ != nullptr && __builtin_amdgcn_mbcnt_hi((uint32_t)(ex_ >> 32),            \
                            __builtin_amdgcn_mbcnt_lo((uint32_t)ex_, 0u)) == 0)      \
      dp_[(ph)] = __builtin_amdgcn_s_memrealtime();                                   \
  } while (0)
#else
#define DSTAMP(ph) \
  do {             \
  } while (0)
#define DSTAMPV(ph, v) \
  do {                 \
  } while (0)
#define DSTAMPA(ph) \
  do {              \
  } while (0)
#define STAMP(ph, val) \
  do {                 \
  } while (0)
#endif

// Sum over each 8-lane group (lanes 8g..8g+7); every lane of the group gets it.
__device__ __forceinline__ uint32_t group_sum8(uint32_t v) {
  v += __builtin_amdgcn_update_dpp(0u, v, 0xb1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
  v += __builtin_amdgcn_update_dpp(0u, v, 0x4e, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
  v += __builtin_amdgcn_update_dpp(0u, v, 0x141, 0xf, 0xf, false);  // row_half_mirror
  return v;
}

// The body stream of the frame (see "Body streaming engine") whose window starts at abase (span window bytes):
// off0 = a0 - abase, in (0, HB], a multiple of 16, and its chunks (the last
// may be partial).
__device__ __forceinline__ uint32_t body_off0(uint64_t abase) {
  return (uint32_t)(((abase + HB) & ~(uint64_t)127) - abase);
}
__device__ __forceinline__ uint32_t body_chunks(uint32_t off0, int span) {
  return span > HB ? ((uint32_t)span - off0 + 15u) >> 4 : 0u;
}

// ---------------------------------------------------------------------------
// Demux: one lookup stage walked to its end (every match counted).

struct Match {
  int32_t first;
  uint32_t n;
};

__device__ __forceinline__ bool occ_bit(const uint32_t* occ, uint32_t i) {
  return ((occ[i >> 5] >> (i & 31u)) & 1u) != 0;
}

// ci_sock_intf_check (netif_table.h:30-36) on the socket fields of a slot;
// hwp is the packet's hwport (lane_hwport), 0xff for none.
__device__ __forceinline__ bool bind2dev_ok(uint32_t sflags, uint64_t hwports, int b2d_vlan,
                                            uint32_t hwp, int vlan) {
  // (bitwise, not short-circuit: no branches in the walks' inner step)
  return !(sflags & OO_GPU_RX_SOCK_BIND2DEV) |
         ((hwp < 64) & (((hwports >> (hwp & 63u)) & 1u) != 0) & (b2d_vlan == vlan));
}

// A slot record as loaded: an IPv4 Slot4 in d0..d1, an IPv6 Slot6 in
// d0..d3 (oo_rx_device.h).
struct Rec {
  uint4 d0, d1, d2, d3;
};

// The table a lane probes.  One wave may hold IPv4 and IPv6 packets; each
// lane walks its own table in the same instruction stream (one chain of
// dependent loads per wave, not one per address family).  The table
// addresses are picked from the (scalar) kernel arguments at each use: held
// per lane they would be loop-invariant VGPRs the kernel cannot afford.
struct Probe {
  uint64_t occ, slots;  // this lane's table (per tile: not loop-invariant)
  uint32_t mask;
  bool is6;
  static constexpr bool kLds = false;
};
// The same with the occupancy bitmaps (and the intf -> hwport bytes) copied
// into the block's LDS (win_kernel): `lo` is the LDS address of this lane's
// family's bitmap.  The bit reads then leave the vector-memory path, whose
// scattered 64-line requests saturate the CU's texture units on short
// frames (TA / TD busy 78 / 95 %, config 3).
struct ProbeL : Probe {
  uint32_t lo;
  static constexpr bool kLds = true;
};

// A kernel-argument value forced into a scalar register: a per-lane select
// between two kernel-argument fields may otherwise be turned into a vector
// load from the argument segment (a memory round trip and a vmcnt(0) drain).
__device__ __forceinline__ uint32_t sreg(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}
__device__ __forceinline__ uint64_t sreg64(const void* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  return (uint64_t)sreg((uint32_t)v) | ((uint64_t)sreg((uint32_t)(v >> 32)) << 32);
}

// Global-address-space loads from an address held as an integer (a plain
// pointer rebuilt from one would be a flat access, counted in lgkmcnt too).
typedef const __attribute__((address_space(1))) uint32_t* g_cu32p;
typedef const __attribute__((address_space(1))) u32x4* g_cu32x4p;
__device__ __forceinline__ uint32_t gload4(uint64_t a) { return *reinterpret_cast<g_cu32p>(a); }
__device__ __forceinline__ uint4 gload16(uint64_t a) {
  const u32x4 v = *reinterpret_cast<g_cu32x4p>(a);
  return make_uint4(v.x, v.y, v.z, v.w);
}
// The same load as an instruction the compiler does not track: the caller
// waits for it with a counted vm_wait before using the value (kx_lookup's
// first level under window_loop's staging).
__device__ __forceinline__ uint4 gload16_untracked(uint64_t a) {
  u32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(a) : "memory");
  return make_uint4(v.x, v.y, v.z, v.w);
}

// A 64-bit per-lane choice between two scalar values, as two 32-bit
// selects (a 64-bit select may become a divergent branch that splits a batch
// of loads).
__device__ __forceinline__ uint64_t sel64(bool c, uint64_t a, uint64_t b) {
  const uint32_t lo = c ? (uint32_t)a : (uint32_t)b, hi = c ? (uint32_t)(a >> 32) : (uint32_t)(b >> 32);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

__device__ __forceinline__ Probe probe_of(const KParams& P, bool is6) {
  Probe t;
  t.is6 = is6;
  t.mask = is6 ? sreg(P.ip6_mask) : sreg(P.ip4_mask);
  t.occ = sel64(is6, sreg64(P.occ6), sreg64(P.occ4));
  t.slots = sel64(is6, sreg64(P.slot6), sreg64(P.slot4));
  return t;
}

// The occupancy words of six slots (every stage's first slot and its
// successor) in one batch: six loads, one wait.  Written as one asm block
// because the register-bound scheduler otherwise consumes each load before
// issuing the next (six memory latencies instead of one).  The wait is
// vmcnt(0): loads complete in issue order and these are the newest, so it
// waits for nothing they would not.
// With them, the lane's byte of the context's intf_i_to_hwport table at
// address ha (netif_table.h:33, in HBM beside the zero region; a per-lane
// index, so a vector load, which here costs no wait of its own -- inside the
// walks its wait would drain the body stream).
__device__ __forceinline__ void occ_words6(const ProbeL& t, const uint32_t i[6], uint32_t w[6],
                                           uint64_t ha, uint32_t& hw) {
  uint32_t a[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) a[k] = t.lo + 4u * (i[k] >> 5);
  asm volatile(
      "ds_read_b32 %0, %7\n\tds_read_b32 %1, %8\n\tds_read_b32 %2, %9\n\t"
      "ds_read_b32 %3, %10\n\tds_read_b32 %4, %11\n\tds_read_b32 %5, %12\n\t"
      "ds_read_u8 %6, %13\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3]), "=&v"(w[4]), "=&v"(w[5]), "=&v"(hw)
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"((uint32_t)ha)
      : "memory");
}
__device__ __forceinline__ void occ_words4(const ProbeL& t, const uint32_t i[4], uint32_t w[4],
                                           uint64_t ha, uint32_t& hw) {
  uint32_t a[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) a[k] = t.lo + 4u * (i[k] >> 5);
  asm volatile(
      "ds_read_b32 %0, %5\n\tds_read_b32 %1, %6\n\tds_read_b32 %2, %7\n\t"
      "ds_read_b32 %3, %8\n\tds_read_u8 %4, %9\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3]), "=&v"(hw)
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"((uint32_t)ha)
      : "memory");
}
__device__ __forceinline__ void occ_words6(const Probe& t, const uint32_t i[6], uint32_t w[6],
                                           uint64_t ha, uint32_t& hw) {
  uint64_t a[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) a[k] = t.occ + 4u * (i[k] >> 5);
  asm volatile(
      "global_load_dword %0, %7, off\n\tglobal_load_dword %1, %8, off\n\t"
      "global_load_dword %2, %9, off\n\tglobal_load_dword %3, %10, off\n\t"
      "global_load_dword %4, %11, off\n\tglobal_load_dword %5, %12, off\n\t"
      "global_load_ubyte %6, %13, off\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3]), "=&v"(w[4]), "=&v"(w[5]), "=&v"(hw)
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(ha)
      : "memory");
}

__device__ __forceinline__ void occ_words4(const Probe& t, const uint32_t i[4], uint32_t w[4],
                                           uint64_t ha, uint32_t& hw) {
  uint64_t a[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) a[k] = t.occ + 4u * (i[k] >> 5);
  asm volatile(
      "global_load_dword %0, %5, off\n\tglobal_load_dword %1, %6, off\n\t"
      "global_load_dword %2, %7, off\n\tglobal_load_dword %3, %8, off\n\t"
      "global_load_ubyte %4, %9, off\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3]), "=&v"(hw)
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(ha)
      : "memory");
}

__device__ __forceinline__ bool probe_occ(const KParams& P, const Probe& t, uint32_t i) {
  (void)P;
  return ((gload4(t.occ + 4u * (i >> 5)) >> (i & 31u)) & 1u) != 0;
}
__device__ __forceinline__ bool probe_occ(const KParams& P, const ProbeL& t, uint32_t i) {
  (void)P;
  uint32_t w;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(w) : "v"(t.lo + 4u * (i >> 5)) : "memory");
  return ((w >> (i & 31u)) & 1u) != 0;
}

template <class PR>
__device__ __forceinline__ Rec load_rec(const KParams& P, const PR& t, uint32_t i, bool any6) {
  (void)P;
  const uint64_t a = t.slots + ((uint64_t)i << (t.is6 ? 6 : 5));
  Rec r;
  r.d0 = gload16(a);
  r.d1 = gload16(a + 16u);
  r.d2 = r.d3 = make_uint4(0, 0, 0, 0);
  if (any6) {
    // No branch (one would end in a wait for the loads above): an IPv4
    // lane reads its first half again and ignores it.
    const uint64_t b = t.is6 ? a + 32u : a;
    r.d2 = gload16(b);
    r.d3 = gload16(b + 16u);
  }
  return r;
}

// One visited slot against the lookup key:
//  IPv4 (handle_entry, netif_table.c:192-231): the first probe matches only
//   an OCCUPIED_PREFERRED entry and its lport is implied (LPRP, hash.h:76-163,
//   :280); later probes match any occupied entry with lport compared;
//   laddr, raddr, rport and protocol always (raddr/rport/protocol are the
//   socket's, ip.h:1315-1340).
//  IPv6 (netif_table_ip6.c:146-170): occupied (id >= 0), laddr, lport,
//   protocol, and either raddr/rport or -- for a wildcard lookup -- a socket
//   that is not connected.
// Then ci_sock_intf_check.  *id is the entry's socket id.
template <bool IS6>
__device__ __forceinline__ bool rec_match(const KParams& P, const Rec& r, bool first4,
                                          const uint32_t la[4], uint32_t lp, const uint32_t ra[4],
                                          bool ra_null, uint32_t rp, uint32_t proto, uint32_t hwp,
                                          int vlan, int32_t& id) {
  bool ok;
  uint32_t sflags;
  int b2d;
  uint64_t hw;
  // (the compares are combined bitwise, not short-circuit: a chain of
  // branches in the walks' inner step costs more than the compares)
  if (!IS6) {
    const uint32_t st = r.d0.x & ST_MASK;
    const bool stok = first4 ? st == ST_PREFERRED : (occupied(st) & ((r.d0.w & 0xffffu) == lp));
    ok = stok & (r.d0.y == la[0]) & (r.d0.z == ra[0]) & ((r.d0.w >> 16) == rp) &
         ((r.d1.x & 0xffu) == proto);
    sflags = r.d1.x >> 16;
    b2d = (int)(int16_t)(r.d1.y & 0xffffu);
    hw = (uint64_t)r.d1.z | ((uint64_t)r.d1.w << 32);
    id = (int32_t)(r.d0.x & ID_MASK);
  } else {
    id = (int32_t)r.d0.x;
    sflags = r.d2.w >> 16;
    const bool rok = ra_null ? !(sflags & OO_GPU_RX_SOCK_CONNECTED)
                             : ((r.d1.z == ra[0]) & (r.d1.w == ra[1]) & (r.d2.x == ra[2]) &
                                (r.d2.y == ra[3]) & ((r.d2.z >> 16) == rp));
    ok = (id >= 0) & (r.d0.z == la[0]) & (r.d0.w == la[1]) & (r.d1.x == la[2]) & (r.d1.y == la[3]) &
         ((r.d2.z & 0xffffu) == lp) & ((r.d2.w & 0xffu) == proto) & rok;
    b2d = (int)(int16_t)(r.d3.x & 0xffffu);
    hw = (uint64_t)r.d3.z | ((uint64_t)r.d3.w << 32);
  }
  (void)P;
  return ok & bind2dev_ok(sflags, hw, b2d, hwp, vlan);
}

// One slot against the lookup key for a lane of either family: M = 0 IPv4,
// 1 IPv6, 2 per lane (t.is6) -- both compares, no loads, so a wave holding
// both families walks in one instruction stream.
template <int M, class PR>
__device__ __forceinline__ bool rec_match_m(const KParams& P, const PR& t, const Rec& r,
                                            bool first4, const uint32_t la[4], uint32_t lp,
                                            const uint32_t ra[4], bool ra_null, uint32_t rp,
                                            uint32_t proto, uint32_t hwp, int vlan, int32_t& id) {
  if (M == 0) return rec_match<false>(P, r, first4, la, lp, ra, ra_null, rp, proto, hwp, vlan, id);
  if (M == 1) return rec_match<true>(P, r, first4, la, lp, ra, ra_null, rp, proto, hwp, vlan, id);
  int32_t id4, id6;
  const bool m4 = rec_match<false>(P, r, first4, la, lp, ra, ra_null, rp, proto, hwp, vlan, id4);
  const bool m6 = rec_match<true>(P, r, first4, la, lp, ra, ra_null, rp, proto, hwp, vlan, id6);
  id = t.is6 ? id6 : id4;
  return t.is6 ? m6 : m4;
}

// ci_netif_filter_for_each_match (netif_table.c:234-319) /
// ci_netif_filter_for_each_match_ip6 (netif_table_ip6.c:110-189) over the
// slot records, every match counted.  The caller has loaded the not-EMPTY
// bits of the first slot (occ) and of the next one on the probe sequence
// (occ_next), and -- when have -- the first slot's record: the common walk
// (an EMPTY first slot, or one occupied slot followed by an EMPTY one) needs
// no more loads.  Tombstones continue the walk; an EMPTY slot or a full
// cycle ends it, and so does the first match when stop: TCP's deliver
// callbacks always return 1 (tcp_rx.c:4644-4657), which ends the reference's
// walk there (handle_entry, netif_table.c:225-229); UDP counts every match
// (ci_udp_rx_deliver continues past a multicast destination or a socket
// that drops, udp_rx.c:194-228).
template <int M, class PR>
__device__ Match walk(const KParams& P, const PR& t, bool any6, const uint32_t la[4],
                      uint32_t lp, const uint32_t ra[4], bool ra_null, uint32_t rp, uint32_t proto,
                      uint32_t hwp, int vlan, uint32_t h1, uint32_t h2, bool occ, Rec rec, bool have,
                      bool occ_next, bool stop) {
  Match m = {-1, 0};
  const uint32_t first = h1;
  if (occ && !have) rec = load_rec(P, t, h1, any6);  // the first slot's record was not preloaded
  for (uint32_t guard = 0; guard <= t.mask; ++guard) {
    if (!occ) break;  // an EMPTY slot ends the walk
    int32_t id;
    if (rec_match_m<M>(P, t, rec, guard == 0, la, lp, ra, ra_null, rp, proto, hwp, vlan, id)) {
      if (m.n == 0) m.first = id;
      ++m.n;
      if (stop) break;
    }
    h1 = (h1 + h2) & t.mask;
    if (h1 == first) break;
    if (guard == 0) {
      occ = occ_next;
      if (occ) rec = load_rec(P, t, h1, any6);
    } else {
      // Deeper in a chain: the record is loaded beside its occupancy bit
      // (one load latency per step, not two; an EMPTY slot's record is
      // simply not used).
      rec = load_rec(P, t, h1, any6);
      occ = probe_occ(P, t, h1);
    }
  }
  return m;
}

// ---------------------------------------------------------------------------
// Header work of one packet (one lane).

// What the parse leaves for the verdict.
struct Parsed {
  oo_gpu_rx_result r;  // the record; final unless the verdict waits for the body
  uint32_t s4;         // window-word sum of the L4 region's bytes in the window,
                       // minus its complement past the window (mod 2^32)
  uint32_t pseudo;     // pseudo-header word sum
  uint32_t odd_long;   // bit 0: odd frame address (RFC 1071 byte swap);
                       // bit 1: the L4 region runs past the window
};

// Window-word sum of window bytes [S, E) read from HBM (the rare L4 region
// that ends before the frame does, past the window).
__device__ __noinline__ uint32_t window_sum_global(uint64_t abase, int S, int E) {
  uint32_t s = 0;
  for (int c = S >> 4; c * 16 < E; ++c) {
    const uint4 v = *reinterpret_cast<const uint4*>(abase + (uint64_t)c * 16);
    s += chunk_sum(v, c * 16, S, E);
  }
  return s;
}

// What the header stage hands the record/demux stage (both parse paths).
struct Hdr {
  uint32_t reason;  // PENDING: the checksums passed (or the L4 verdict waits for the body)
  uint32_t late;    // PENDING, or why a packet that passed them is dropped (IPv4 only)
  uint32_t flags;   // OO_RX_F_VLAN / OO_RX_F_IP6
  uint32_t vlan, proto, ip_paylen, l4;
  bool l3ok, is6, longl4;
  uint32_t sport, dport;  // network order in host integers
  uint32_t sa[4], da[4];  // IPv6 addresses, or the IPv4 ones in [0]
  uint32_t s4, pseudo;
  int E4;
};

// A packet's staged window in LDS (stage_window): a 128-B row whose 16-B
// cell k sits at row + 16 * ((k + rot) & 7).
struct Win {
  const uint8_t* row;
  uint32_t rot;
  __device__ __forceinline__ const uint8_t* cell(int k) const {
    return row + ((((uint32_t)k + rot) & 7u) << 4);
  }
};

// The staged window of this lane's packet in registers (one LDS wait).
__device__ __forceinline__ void read_cells(const Win& W, uint4 (&c)[HC]) {
  static_assert(HC == 8, "eight window cells");
  uint32_t a[HC];
#pragma unroll
  for (int k = 0; k < HC; ++k) a[k] = (uint32_t)(uintptr_t)(lptr)(W.cell(k));
  asm volatile(
      "ds_read_b128 %0, %8\n\tds_read_b128 %1, %9\n\t"
      "ds_read_b128 %2, %10\n\tds_read_b128 %3, %11\n\t"
      "ds_read_b128 %4, %12\n\tds_read_b128 %5, %13\n\t"
      "ds_read_b128 %6, %14\n\tds_read_b128 %7, %15\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(c[0]), "=&v"(c[1]), "=&v"(c[2]), "=&v"(c[3]), "=&v"(c[4]), "=&v"(c[5]),
        "=&v"(c[6]), "=&v"(c[7])
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7])
      : "memory");
}

// The eight cells and two more (by address) in one batch with one wait.
__device__ __forceinline__ void read_cells_and(const Win& W, uint32_t ah, uint32_t at, uint4 (&c)[HC],
                                               uint4& ch, uint4& ct) {
  uint32_t a[HC];
#pragma unroll
  for (int k = 0; k < HC; ++k) a[k] = (uint32_t)(uintptr_t)(lptr)(W.cell(k));
  asm volatile(
      "ds_read_b128 %0, %10\n\tds_read_b128 %1, %11\n\t"
      "ds_read_b128 %2, %12\n\tds_read_b128 %3, %13\n\t"
      "ds_read_b128 %4, %14\n\tds_read_b128 %5, %15\n\t"
      "ds_read_b128 %6, %16\n\tds_read_b128 %7, %17\n\t"
      "ds_read_b128 %8, %18\n\tds_read_b128 %9, %19\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(c[0]), "=&v"(c[1]), "=&v"(c[2]), "=&v"(c[3]), "=&v"(c[4]), "=&v"(c[5]),
        "=&v"(c[6]), "=&v"(c[7]), "=&v"(ch), "=&v"(ct)
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]),
        "v"(ah), "v"(at)
      : "memory");
}

// Word sum of the cell's words whose bits are set in wm (8 bits).
__device__ __forceinline__ uint32_t cell_sum_masked(const uint4& v, uint32_t wm, uint32_t acc) {
  auto wt = [&](int i) { return ((wm >> (2 * i)) & 1u) | (((wm >> (2 * i + 1)) & 1u) << 16); };
  acc = dot(v.x, wt(0), acc);
  acc = dot(v.y, wt(1), acc);
  acc = dot(v.z, wt(2), acc);
  return dot(v.w, wt(3), acc);
}

// Byte b (0..15) of a cell.
__device__ __forceinline__ uint32_t cell_byte(const uint4& v, uint32_t b) {
  const uint32_t i = b >> 2;
  const uint32_t w = i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w;
  return (w >> (8 * (b & 3u))) & 0xffu;
}

// The partial-cell part of a window-word sum of window bytes [lo, hi)
// (0 <= lo <= hi <= HB) -- words pair at even window positions: the words
// [wlo, whi) of the head cell kh and the tail cell kt (their bytes in ch, ct),
// an odd end's half word taken off; the cells strictly between are the
// caller's (whole).
struct WinSpan {
  uint32_t wlo, whi, kh, kt;
  bool any;
};
__device__ __forceinline__ WinSpan win_span(int lo, int hi) {
  WinSpan w;
  w.wlo = (uint32_t)lo >> 1;
  w.whi = (uint32_t)(hi + 1) >> 1;
  w.any = w.wlo < w.whi;
  w.kh = w.wlo >> 3;
  w.kt = w.any ? (w.whi - 1u) >> 3 : w.kh;
  return w;
}
__device__ __forceinline__ uint32_t win_span_ends(const WinSpan& w, int lo, int hi, const uint4& ch,
                                                  const uint4& ct, uint32_t s) {
  const uint32_t a = w.wlo & 7u;
  const uint32_t bh = w.kh == w.kt ? w.whi - 8u * w.kh : 8u;
  s = cell_sum_masked(ch, w.any ? ((1u << bh) - 1u) & ~((1u << a) - 1u) : 0u, s);
  s = cell_sum_masked(ct, w.any && w.kt != w.kh ? (1u << (w.whi - 8u * w.kt)) - 1u : 0u, s);
  if (lo & 1) s -= cell_byte(ch, (uint32_t)(lo - 1) & 15u);
  if (hi & 1) s -= cell_byte(ct, (uint32_t)hi & 15u) << 8;
  return s;
}

// The whole window-word sum of [lo, hi): what chunk_sum gives summed over
// the eight cells (read here with the two end cells, one batch).
__device__ __forceinline__ uint32_t window_sum(const Win& W, int lo, int hi) {
  const WinSpan w = win_span(lo, hi);
  uint4 c[HC], ch, ct;
  read_cells_and(W, (uint32_t)(uintptr_t)(lptr)(W.cell((int)(w.kh & 7u))),
                 (uint32_t)(uintptr_t)(lptr)(W.cell((int)(w.kt & 7u))), c, ch, ct);
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < HC; ++k) {
    const uint32_t t = chunk_sum_all(c[k], 0u);
    s += ((uint32_t)k > w.kh && (uint32_t)k < w.kt) ? t : 0u;
  }
  return win_span_ends(w, lo, hi, ch, ct, s);
}

// The same from cells already in registers (the end cells read again from
// LDS: a register array indexed per lane would go through scratch); only
// cells from KMIN on can lie inside.
template <int KMIN>
__device__ __forceinline__ uint32_t window_sum_cells(const Win& W, const uint4 (&c)[HC], int lo, int hi) {
  const WinSpan w = win_span(lo, hi);
  uint4 ch, ct;
  {
    const uint32_t ah = (uint32_t)(uintptr_t)(lptr)(W.cell((int)(w.kh & 7u)));
    const uint32_t at = (uint32_t)(uintptr_t)(lptr)(W.cell((int)(w.kt & 7u)));
    asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %3\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(ch), "=&v"(ct)
                 : "v"(ah), "v"(at)
                 : "memory");
  }
  uint32_t s = 0;
#pragma unroll
  for (int k = KMIN; k < HC; ++k) {
    const bool in = (uint32_t)k > w.kh && (uint32_t)k < w.kt;
    if (__ballot(in) != 0) s += in ? chunk_sum_all(c[k], 0u) : 0u;  // (short regions: no lane)
  }
  return win_span_ends(w, lo, hi, ch, ct, s);
}

// Window bytes q and q + 1 (q + 1 < HB), low half: two byte reads, one wait.
__device__ __forceinline__ uint32_t win_byte_pair(const Win& W, uint32_t q) {
  const uint32_t row = (uint32_t)(uintptr_t)(lptr)(W.row);
  const uint32_t r = q + 1u;
  const uint32_t a0 = row + ((((q >> 4) + W.rot) & 7u) << 4) + (q & 15u);
  const uint32_t a1 = row + ((((r >> 4) + W.rot) & 7u) << 4) + (r & 15u);
  uint32_t b0, b1;
  asm volatile("ds_read_u8 %0, %2\n\tds_read_u8 %1, %3\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(b0), "=&v"(b1)
               : "v"(a0), "v"(a1)
               : "memory");
  return b0 | (b1 << 8);
}

// K aligned 4-byte LDS reads in one batch with one wait.
template <int K>
__device__ __forceinline__ void lds_read_b32s(const uint32_t (&a)[K], uint32_t (&d)[K]);
template <>
__device__ __forceinline__ void lds_read_b32s<7>(const uint32_t (&a)[7], uint32_t (&d)[7]) {
  asm volatile("ds_read_b32 %0, %7\n\tds_read_b32 %1, %8\n\tds_read_b32 %2, %9\n\tds_read_b32 %3, %10\n\tds_read_b32 %4, %11\n\tds_read_b32 %5, %12\n\tds_read_b32 %6, %13\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(d[0]), "=&v"(d[1]), "=&v"(d[2]), "=&v"(d[3]), "=&v"(d[4]), "=&v"(d[5]), "=&v"(d[6])
               : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6])
               : "memory");
}
template <>
__device__ __forceinline__ void lds_read_b32s<11>(const uint32_t (&a)[11], uint32_t (&d)[11]) {
  asm volatile("ds_read_b32 %0, %11\n\tds_read_b32 %1, %12\n\tds_read_b32 %2, %13\n\tds_read_b32 %3, %14\n\tds_read_b32 %4, %15\n\tds_read_b32 %5, %16\n\tds_read_b32 %6, %17\n\tds_read_b32 %7, %18\n\tds_read_b32 %8, %19\n\tds_read_b32 %9, %20\n\tds_read_b32 %10, %21\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(d[0]), "=&v"(d[1]), "=&v"(d[2]), "=&v"(d[3]), "=&v"(d[4]), "=&v"(d[5]), "=&v"(d[6]), "=&v"(d[7]), "=&v"(d[8]), "=&v"(d[9]), "=&v"(d[10])
               : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]), "v"(a[8]), "v"(a[9]), "v"(a[10])
               : "memory");
}
template <>
__device__ __forceinline__ void lds_read_b32s<13>(const uint32_t (&a)[13], uint32_t (&d)[13]) {
  asm volatile("ds_read_b32 %0, %13\n\tds_read_b32 %1, %14\n\tds_read_b32 %2, %15\n\tds_read_b32 %3, %16\n\tds_read_b32 %4, %17\n\tds_read_b32 %5, %18\n\tds_read_b32 %6, %19\n\tds_read_b32 %7, %20\n\tds_read_b32 %8, %21\n\tds_read_b32 %9, %22\n\tds_read_b32 %10, %23\n\tds_read_b32 %11, %24\n\tds_read_b32 %12, %25\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(d[0]), "=&v"(d[1]), "=&v"(d[2]), "=&v"(d[3]), "=&v"(d[4]), "=&v"(d[5]), "=&v"(d[6]), "=&v"(d[7]), "=&v"(d[8]), "=&v"(d[9]), "=&v"(d[10]), "=&v"(d[11]), "=&v"(d[12])
               : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]), "v"(a[8]), "v"(a[9]), "v"(a[10]), "v"(a[11]), "v"(a[12])
               : "memory");
}

// Frame bytes [j0, j0 + 4 (K - 1)) of this lane's window (frame byte j at
// window position shift + j) as K - 1 little-endian words: K aligned reads
// from window position (shift + j0) & ~3 on, one batch, realigned (a word
// never straddles a cell; a position past the window wraps inside the row
// and is only ever read for bytes nothing uses).
template <int K>
__device__ __forceinline__ void window_run(const Win& W, int shift, int j0, uint32_t (&o)[K - 1]) {
  const uint32_t p = (uint32_t)(shift + j0);
  const uint32_t row = (uint32_t)(uintptr_t)(lptr)(W.row);
  uint32_t a[K], d[K];
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const uint32_t q = (p & ~3u) + 4u * (uint32_t)i;
    a[i] = row + ((((q >> 4) + W.rot) & 7u) << 4) + (q & 12u);
  }
  lds_read_b32s<K>(a, d);
#pragma unroll
  for (int i = 0; i < K - 1; ++i) o[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], p & 3u);
}

// (A per-lane select by lane mask: the compiler turns a select between
// neighbouring array elements into an indexed access through scratch.)
__device__ __forceinline__ uint32_t vsel(uint64_t m, uint32_t if0, uint32_t if1) {
  uint32_t r;
  asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(if0), "v"(if1), "s"(m));
  return r;
}

// Bit i: option byte i is not IPOPT_NOP (bytes 0..39).
__device__ __forceinline__ uint64_t opt_not_nop(const uint32_t (&O)[10]) {
  uint64_t m = 0;
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    const uint32_t x = O[k] ^ 0x01010101u;
    // bit 7 of each byte: the byte is non-zero; gathered to bits 28..31
    const uint32_t y = (((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
    m |= (uint64_t)((y * 0x00204081u) >> 28) << (4 * k);
  }
  return m;
}

#ifndef OO_RX_GEN_RUNS  // the general header walk by word runs (parse_general_runs)
#define OO_RX_GEN_RUNS 1
#endif
// The general header walk by runs (OO_RX_GEN_RUNS): the same decisions as
// parse_general below in fewer instructions -- config 4's win_kernel issues
// instructions most of the time, and its walk was 13 of 22 us per tile
// (stamps).  Fields come from a few word runs of the window, each one batch
// of LDS reads (frame bytes 12..63: Ethernet type, VLAN tag and the L3
// header at either place; the L4 header's first 24 bytes; the IPv4
// options); the IPv4 header sum from those words (frame-aligned pairs: the
// folded sum is the window-aligned one byte-swapped, and 0xffff either
// way, RFC 1071); the option walk steps from one non-NOP byte to the next.
__device__ __forceinline__ Hdr parse_general_runs(const Win& W, int shift, int len, int off0) {
  // Frame bytes [12, 60).  Only bytes 12..15 can lie past the frame and
  // still be used (the VLAN tag is recorded for any length): masked.
  uint32_t F[12];
  window_run<13>(W, shift, 12, F);
  {
    const int nv = len - 12;
    F[0] &= nv >= 4 ? 0xffffffffu : nv <= 0 ? 0u : (1u << (8 * nv)) - 1u;
  }
  auto bF = [&](int i) -> uint32_t { return (F[i >> 2] >> (8 * (i & 3))) & 0xffu; };  // byte 12 + i
  auto BE16F = [&](int i) -> uint32_t { return (bF(i) << 8) | bF(i + 1); };

  Hdr h;
  h.flags = 0;
  h.late = PENDING;
  const bool vl = BE16F(0) == 0x8100u;  // ci_parse_rx_vlan (netif_event.c:116-132)
  const int pre_l3 = vl ? 18 : 14;
  h.vlan = vl ? BE16F(2) & 0xfffu : 0u;
  if (vl) h.flags |= OO_RX_F_VLAN;
  // The L3 header's first 40 bytes: L[k] = frame bytes l3 + 4k .. l3 + 4k + 3.
  uint32_t L[10];
#pragma unroll
  for (int k = 0; k < 10; ++k)
    L[k] = vl ? __builtin_amdgcn_alignbyte(F[k + 2], F[k + 1], 2u)
              : __builtin_amdgcn_alignbyte(F[k + 1], F[k], 2u);
  auto bL = [&](int i) -> uint32_t { return (L[i >> 2] >> (8 * (i & 3))) & 0xffu; };
  auto BE16L = [&](int i) -> uint32_t { return (bL(i) << 8) | bL(i + 1); };
  auto N16L = [&](int i) -> uint32_t { return (L[i >> 2] >> (8 * (i & 3))) & 0xffffu; };  // i even

  const int l3 = pre_l3;
  uint32_t reason = PENDING;
  bool is6 = false, l3ok = false;
  int ip_len = 0, ihl4 = 0, ip_paylen = 0, l4 = 0;
  uint32_t proto = 0;
  if (len < pre_l3 + 20) {  // netif_event.c:1030
    reason = OO_RX_R_SHORT_L2;
  } else {
    const uint32_t et = vl ? BE16F(4) : BE16F(0);
    if (et == 0x0800u) {  // :1038-1058
      l3ok = true;
      ip_len = (int)BE16L(2);
      ihl4 = (int)(bL(0) & 0xfu) * 4;
      ip_paylen = ip_len - ihl4;
      proto = bL(9);
      if (ip_paylen <= 0 || len < pre_l3 + ip_len) reason = OO_RX_R_IP4_LEN;
      l4 = l3 + ihl4;
    } else if (et == 0x86ddu) {  // :1060-1076
      l3ok = true;
      is6 = true;
      h.flags |= OO_RX_F_IP6;
      ip_paylen = (int)BE16L(4);
      proto = bL(6);
      if (ip_paylen <= 0 || len < pre_l3 + 40 + ip_paylen) reason = OO_RX_R_IP6_LEN;
      l4 = l3 + 40;
    } else {
      reason = OO_RX_R_NOT_IP;  // :1078
    }
  }
  DSTAMPA(9);

  // Frame bytes [l4, l4 + 24): every field read from them is inside the
  // frame whenever it is used (the gates come first).
  uint32_t G[6];
  window_run<7>(W, shift, l4, G);
  auto bG = [&](int i) -> uint32_t { return (G[i >> 2] >> (8 * (i & 3))) & 0xffu; };
  auto N16G = [&](int i) -> uint32_t { return (G[i >> 2] >> (8 * (i & 3))) & 0xffffu; };  // i even
  // The IPv4 options, bytes [l3 + 20, l3 + 60), when some lane has any.
  const int nopt = l3ok && !is6 && ihl4 > 20 ? (ihl4 - 20) >> 2 : 0;  // option words
  uint32_t O[10];
  if (__ballot(nopt != 0) != 0) {
    window_run<11>(W, shift, l3 + 20, O);
  } else {
#pragma unroll
    for (int k = 0; k < 10; ++k) O[k] = 0u;
  }

  // L4 gates (netif_event.c:1084-1127) -> which region to sum.
  uint32_t l4_gate = PENDING;
  bool need_l4 = false;
  int l4_len = 0;
  uint32_t pseudo = 0;
  if (reason == PENDING) {
    if (proto == 6u) {
      const int hlen = (int)((bG(12) & 0xf0u) >> 2);
      if (ip_paylen < 20) l4_gate = OO_RX_R_TCP_SHORT;
      else if (hlen < 20 || ip_paylen < hlen) l4_gate = OO_RX_R_TCP_CSUM;
      else { need_l4 = true; l4_len = ip_paylen; }
    } else if (proto == 17u) {
      const uint32_t udp_len = swap16(N16G(4));
      if (ip_paylen < 8) l4_gate = OO_RX_R_UDP_SHORT;
      else if (udp_len < 8u || udp_len > (uint32_t)ip_paylen) l4_gate = OO_RX_R_UDP_CSUM;
      else if (!(N16G(6) == 0u && !is6)) { need_l4 = true; l4_len = (int)udp_len; }
    } else {
      l4_gate = OO_RX_R_PROTO_OTHER;
    }
    if (need_l4) {
      // Pseudo-header words (checksum.c:215-223, 304-305, 334-335).
      if (is6) {
        uint32_t a = 0;
#pragma unroll
        for (int k = 2; k < 10; ++k) a = dot(L[k], 0x00010001u, a);
        pseudo = a + (proto == 6u ? N16L(4) + 0x0600u : N16G(4) + 0x1100u);
      } else {
        pseudo = dot(L[4], 0x00010001u, dot(L[3], 0x00010001u, 0u));
        if (proto == 6u) {
          const uint32_t pl = (uint32_t)ip_paylen & 0xffffu;
          pseudo += 0x0600u + (((pl & 0xffu) << 8) | (pl >> 8));
        } else {
          pseudo += 0x1100u + N16G(4);
        }
      }
    }
  }
  DSTAMPA(10);

  // The IPv4 header's word sum (its 20 bytes and the option words), and the
  // L4 region's window part over the cells: [S4,E4) when it ends inside the
  // window, else [S4,off0) (signed: the body stream starts at window byte
  // off0, which may lie before S4).
  const bool need_ip = reason == PENDING && !is6;
  const int S4 = shift + l4, E4 = need_l4 ? shift + l4 + l4_len : S4;
  const int cut = E4 > HB ? off0 : E4;
  const int lo4 = min(S4, cut), hi4 = max(S4, cut);
  uint32_t s3 = 0, s4 = 0;
  if (need_ip) {
#pragma unroll
    for (int k = 0; k < 5; ++k) s3 = dot(L[k], 4 * k < ihl4 ? 0x00010001u : 0u, s3);  // (IHL < 5 too)
#pragma unroll
    for (int k = 0; k < 10; ++k) s3 = dot(O[k], k < nopt ? 0x00010001u : 0u, s3);
  }
  if (need_l4) {
    s4 = window_sum(W, lo4, hi4);
    if (cut < S4) s4 = 0u - s4;
  }
  if (reason == PENDING && need_ip) {
    // IHL != 0 makes the word sum non-zero: fold == 0xffff <=> valid.
    if (ihl4 == 0 || fold16(s3) != 0xffffu) reason = OO_RX_R_IP4_CSUM;
  }
  if (reason == PENDING && l4_gate != PENDING) reason = l4_gate;

  // L4 verdict now when the region ends inside the window; otherwise it
  // waits for the body stream and the record is speculative.
  const bool longl4 = reason == PENDING && need_l4 && E4 > HB;
  if (reason == PENDING && need_l4 && !longl4) {
    uint32_t f = fold16(s4);
    if (shift & 1) f = swap16(f);  // RFC 1071 byte-order swap
    if (fold16(f + pseudo) != 0xffffu)
      reason = proto == 6u ? OO_RX_R_TCP_CSUM : OO_RX_R_UDP_CSUM;
  }

  // The TCP timestamp-option fast layout (tcp_rx.c:4537-4543).
  if (reason == PENDING && proto == 6u && bG(12) == 0x80u && G[5] == 0x0a080101u)
    h.flags |= OO_RX_F_TSO;
  DSTAMPA(11);
  h.reason = reason;
  h.proto = proto;
  h.ip_paylen = (uint32_t)ip_paylen;
  h.l4 = (uint32_t)l4;
  h.l3ok = l3ok;
  h.is6 = is6;
  h.longl4 = longl4;
  h.s4 = s4;
  h.pseudo = pseudo;
  h.E4 = E4;
  h.sport = h.dport = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) h.sa[i] = h.da[i] = 0;
  if (reason == PENDING) {
    h.sport = N16G(0);
    h.dport = N16G(2);
    if (is6) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        h.sa[i] = L[2 + i];
        h.da[i] = L[6 + i];
      }
    } else {
      h.sa[0] = L[3];
      h.da[0] = L[4];
      const uint32_t frag = BE16L(6);
      uint32_t late = PENDING;
      DSTAMPA(12);
      if ((frag & 0x3fffu) != 0 || ip_len > len - pre_l3) {
        late = OO_RX_R_IP4_FRAG;  // netif_event.c:293-295
      } else if (ihl4 > 20) {
        // ci_ip_options_parse (netif_event.c:135-185), signed-char lengths:
        // from one non-NOP byte to the next (a NOP only ever advances one
        // byte); a step past the options' end, or onto IPOPT_EOL, ends it.
        const uint64_t nn = opt_not_nop(O);
        const int end = ihl4 - 20;
        int o = 0;
        bool err = false;
        for (;;) {
          const uint64_t rest = nn >> o;
          o += rest != 0 ? (int)__builtin_ctzll(rest) : 64;
          if (o >= end) break;
          const uint32_t b2 = win_byte_pair(W, (uint32_t)(shift + l3 + 20 + o));
          const uint32_t kind = b2 & 0xffu;
          if (kind == 0u) break;  // IPOPT_EOL
          if (kind == 7u || kind == 68u || kind == 130u || kind == 136u) {
            const int l = (int)(int8_t)(uint8_t)(b2 >> 8);
            if (l < 4 || l > end - o) { err = true; break; }
            o += l;
            if (o >= end) break;
          } else {
            err = true;
            break;
          }
        }
        if (err) late = OO_RX_R_IP4_OPTS_BAD;
      }
      if (late == PENDING && proto == 6u && frag != 0x4000u && frag != 0u)
        late = OO_RX_R_TCP_SCATTERED;  // tcp_rx.c:4696-4699
      h.late = late;
    }
  }
  return h;
}

// The general header walk (any VLAN / IP version / IHL / options / alignment)
// over the staged window: handle_rx_csum_bad (netif_event.c:1024-1127) and
// the IPv4 checks of handle_rx_pkt (:293-303, tcp_rx.c:4696-4699).  Window
// byte w is the frame's 16-B-aligned start + w.
__device__ __forceinline__ Hdr parse_general(const Win& W, int shift, int len, int off0) {
  // Header byte j (j >= 0); bytes at or beyond the frame length read 0.
  auto B = [&](int j) -> uint32_t {
    int w = shift + j;
    w = w < HB ? w : HB - 1;
    const uint32_t v = W.cell(w >> 4)[w & 15];
    return j < len ? v : 0u;
  };
  auto BE16 = [&](int j) -> uint32_t { return (B(j) << 8) | B(j + 1); };
  auto N16 = [&](int j) -> uint32_t { return B(j) | (B(j + 1) << 8); };
  auto N32 = [&](int j) -> uint32_t { return N16(j) | (N16(j + 2) << 16); };
  // Window bytes j .. j+3 as a little-endian word, unmasked (two aligned
  // 4-B LDS reads inside the window).
  auto D4 = [&](int j) -> uint32_t {
    int w = shift + j;
    w = w < HB - 4 ? w : HB - 4;
    const int d = w >> 2;
    const uint32_t lo = *reinterpret_cast<const uint32_t*>(W.cell(d >> 2) + 4 * (d & 3));
    const int e = d + 1 < HB / 4 ? d + 1 : d;
    const uint32_t hi = *reinterpret_cast<const uint32_t*>(W.cell(e >> 2) + 4 * (e & 3));
    return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(w & 3));
  };

  Hdr h;
  h.flags = 0;
  h.late = PENDING;
  int pre_l3 = 14;
  h.vlan = 0;
  if (BE16(12) == 0x8100u) {  // ci_parse_rx_vlan (netif_event.c:116-132)
    pre_l3 = 18;
    h.vlan = BE16(14) & 0xfffu;
    h.flags |= OO_RX_F_VLAN;
  }
  const int l3 = pre_l3;
  uint32_t reason = PENDING;
  bool is6 = false, l3ok = false;
  int ip_len = 0, ihl4 = 0, ip_paylen = 0, l4 = 0;
  uint32_t proto = 0;
  if (len < pre_l3 + 20) {  // netif_event.c:1030
    reason = OO_RX_R_SHORT_L2;
  } else {
    const uint32_t et = BE16(pre_l3 - 2);
    if (et == 0x0800u) {  // :1038-1058
      l3ok = true;
      ip_len = (int)BE16(l3 + 2);
      ihl4 = (int)(B(l3) & 0xfu) * 4;
      ip_paylen = ip_len - ihl4;
      proto = B(l3 + 9);
      if (ip_paylen <= 0 || len < pre_l3 + ip_len) reason = OO_RX_R_IP4_LEN;
      l4 = l3 + ihl4;
    } else if (et == 0x86ddu) {  // :1060-1076
      l3ok = true;
      is6 = true;
      h.flags |= OO_RX_F_IP6;
      ip_paylen = (int)BE16(l3 + 4);
      proto = B(l3 + 6);
      if (ip_paylen <= 0 || len < pre_l3 + 40 + ip_paylen) reason = OO_RX_R_IP6_LEN;
      l4 = l3 + 40;
    } else {
      reason = OO_RX_R_NOT_IP;  // :1078
    }
  }
  DSTAMPA(9);

  // L4 gates (netif_event.c:1084-1127) -> which region to sum.
  uint32_t l4_gate = PENDING;
  bool need_l4 = false;
  int l4_len = 0;
  uint32_t pseudo = 0;
  if (reason == PENDING) {
    if (proto == 6u) {
      const int hlen = (int)((B(l4 + 12) & 0xf0u) >> 2);
      if (ip_paylen < 20) l4_gate = OO_RX_R_TCP_SHORT;
      else if (hlen < 20 || ip_paylen < hlen) l4_gate = OO_RX_R_TCP_CSUM;
      else { need_l4 = true; l4_len = ip_paylen; }
    } else if (proto == 17u) {
      const uint32_t udp_len = BE16(l4 + 4);
      if (ip_paylen < 8) l4_gate = OO_RX_R_UDP_SHORT;
      else if (udp_len < 8u || udp_len > (uint32_t)ip_paylen) l4_gate = OO_RX_R_UDP_CSUM;
      else if (!(N16(l4 + 6) == 0u && !is6)) { need_l4 = true; l4_len = (int)udp_len; }
    } else {
      l4_gate = OO_RX_R_PROTO_OTHER;
    }
    if (need_l4) {
      // Pseudo-header words (checksum.c:215-223, 304-305, 334-335).
      if (is6) {
        uint32_t a = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) a += N16(l3 + 8 + 2 * i);
        pseudo = a + (proto == 6u ? N16(l3 + 4) + 0x0600u : N16(l4 + 4) + 0x1100u);
      } else {
        pseudo = N16(l3 + 12) + N16(l3 + 14) + N16(l3 + 16) + N16(l3 + 18);
        if (proto == 6u) {
          const uint32_t pl = (uint32_t)ip_paylen & 0xffffu;
          pseudo += 0x0600u + (((pl & 0xffu) << 8) | (pl >> 8));
        } else {
          pseudo += 0x1100u + N16(l4 + 4);
        }
      }
    }
  }
  DSTAMPA(10);

  // Sums over the staged window: IPv4 header [S3,E3); the L4 region's
  // window part: [S4,E4) when it ends inside the window, else [S4,off0)
  // (signed: the body stream starts at window byte off0, which may lie
  // before S4).
  const bool need_ip = reason == PENDING && !is6;
  const int S3 = shift + l3, E3 = need_ip ? shift + l3 + ihl4 : S3;
  const int S4 = shift + l4, E4 = need_l4 ? shift + l4 + l4_len : S4;
  const int cut = E4 > HB ? off0 : E4;
  const int lo4 = min(S4, cut), hi4 = max(S4, cut);
  uint32_t s3 = 0, s4 = 0;
#ifdef OO_RX_BOUND_NOGENSUM  // (timing bound, wrong records: no window sums in the general walk;
  s3 = 0xffffu;              //  the IPv4 check passes, so the same packets reach the lookups
  if (false) {               //  and the same bodies stream)
#else
  if (need_ip || need_l4) {
#endif
#pragma unroll
    for (int k = 0; k < HC; ++k) {
      const uint4 v = *reinterpret_cast<const uint4*>(W.cell(k));
      if (k * 16 < E3) s3 += chunk_sum(v, k * 16, S3, E3);
      if (k * 16 < hi4) s4 += chunk_sum(v, k * 16, lo4, hi4);
    }
    if (cut < S4) s4 = 0u - s4;
  }
  DSTAMPA(11);
  if (reason == PENDING && need_ip) {
    // IHL != 0 makes the word sum non-zero: fold == 0xffff <=> valid.
    if (ihl4 == 0 || fold16(s3) != 0xffffu) reason = OO_RX_R_IP4_CSUM;
  }
  if (reason == PENDING && l4_gate != PENDING) reason = l4_gate;

  // L4 verdict now when the region ends inside the window; otherwise it
  // waits for the body stream and the record is speculative.
  const bool longl4 = reason == PENDING && need_l4 && E4 > HB;
  if (reason == PENDING && need_l4 && !longl4) {
    uint32_t f = fold16(s4);
    if (shift & 1) f = swap16(f);  // RFC 1071 byte-order swap
    if (fold16(f + pseudo) != 0xffffu)
      reason = proto == 6u ? OO_RX_R_TCP_CSUM : OO_RX_R_UDP_CSUM;
  }

  // The TCP timestamp-option fast layout (tcp_rx.c:4537-4543).
  if (reason == PENDING && proto == 6u && B(l4 + 12) == 0x80u && N32(l4 + 20) == 0x0a080101u)
    h.flags |= OO_RX_F_TSO;
  h.reason = reason;
  h.proto = proto;
  h.ip_paylen = (uint32_t)ip_paylen;
  h.l4 = (uint32_t)l4;
  h.l3ok = l3ok;
  h.is6 = is6;
  h.longl4 = longl4;
  h.s4 = s4;
  h.pseudo = pseudo;
  h.E4 = E4;
  h.sport = h.dport = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) h.sa[i] = h.da[i] = 0;
  if (reason == PENDING) {
    h.sport = N16(l4);
    h.dport = N16(l4 + 2);
    if (is6) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        h.sa[i] = N32(l3 + 8 + 4 * i);
        h.da[i] = N32(l3 + 24 + 4 * i);
      }
    } else {
      h.sa[0] = N32(l3 + 12);
      h.da[0] = N32(l3 + 16);
      const uint32_t frag = BE16(l3 + 6);
      uint32_t late = PENDING;
      if ((frag & 0x3fffu) != 0 || ip_len > len - pre_l3) {
        late = OO_RX_R_IP4_FRAG;  // netif_event.c:293-295
      } else if (ihl4 > 20) {
        // ci_ip_options_parse (netif_event.c:135-185), signed-char lengths.
        // Four option bytes per step: a run of NOPs at the front is taken
        // whole (a run that reaches the end of the options ends the walk,
        // as the byte-at-a-time loop would), else one option.  Bytes read at
        // or past `end` only ever end the walk, so they need no masking.
        int o = l3 + 20;
        const int end = l3 + ihl4;
        bool err = false;
        while (o < end && !err) {
          const uint32_t b4 = D4(o);
          const uint32_t kind = b4 & 0xffu;
          if (kind == 0u) break;  // IPOPT_EOL
          if (kind == 1u) {       // IPOPT_NOP run: count the leading 0x01 bytes
            const uint32_t x = b4 ^ 0x01010101u;
            const uint32_t nz = (x & 0xffu ? 1u : 0u) | (x & 0xff00u ? 2u : 0u) |
                                (x & 0xff0000u ? 4u : 0u) | (x & 0xff000000u ? 8u : 0u);
            o += nz ? (int)__builtin_ctz(nz) : 4;
          } else if (kind == 7u || kind == 68u || kind == 130u || kind == 136u) {
            const int l = (int)(int8_t)(uint8_t)(b4 >> 8);
            if (l < 4 || l > end - o) err = true;
            else o += l;
          } else {
            err = true;
          }
        }
        if (err) late = OO_RX_R_IP4_OPTS_BAD;
      }
      if (late == PENDING && proto == 6u && frag != 0x4000u && frag != 0u)
        late = OO_RX_R_TCP_SCATTERED;  // tcp_rx.c:4696-4699
      h.late = late;
    }
  }
  DSTAMPA(12);
  return h;
}

__device__ __forceinline__ uint32_t bswap16(uint32_t v) { return ((v & 0xffu) << 8) | ((v >> 8) & 0xffu); }

// The fixed-format header (the common frame): 16-B-aligned start, untagged
// Ethernet, IPv4 with IHL 5, not fragmented, TCP or UDP whose length fields
// pass the gates.  Every field sits at a fixed window offset, so it comes out
// of the eight staged cells c[] (window bytes 16k..16k+15 in c[k]) with
// shifts; the same decisions as parse_general for these frames.  Returns
// false (h untouched beyond scratch) for every other frame.
#ifndef OO_RX_FIXED_SPAN
#define OO_RX_FIXED_SPAN 1
#endif
// SPAN: a region ending inside a cell is summed as one span (the cells
// between whole, the end cells masked: window_sum_cells) instead of cell by
// cell (win_kernel; rx_kernel is at its register limit).
template <bool SPAN>
__device__ __forceinline__ bool parse_fixed(const Win& W, const uint4 (&c)[HC], int shift, int len,
                                            int off0, Hdr& h) {
  const uint32_t ip_len = bswap16(c[1].x);
  const uint32_t frag = bswap16(c[1].y);
  const uint32_t proto = c[1].y >> 24;
  const int ip_paylen = (int)ip_len - 20;
  const uint32_t udp_len = bswap16(c[2].y >> 16);
  const int hlen = (int)(((c[2].w >> 16) & 0xf0u) >> 2);
  // (gates combined bitwise: one branch, not one per test)
  const bool tcp = proto == 6u;
  const bool ok = (shift == 0) & (off0 >= 48) & (len >= 48) &
                  ((c[0].w & 0x000fffffu) == 0x00050008u) & (ip_paylen > 0) &
                  (len >= 14 + (int)ip_len) & ((frag & 0x3fffu) == 0u) &
                  (tcp ? ((ip_paylen >= 20) & (hlen >= 20) & (ip_paylen >= hlen))
                       : ((proto == 17u) & (ip_paylen >= 8) & (udp_len >= 8u) &
                          (udp_len <= (uint32_t)ip_paylen)));
  if (!ok) return false;
  const uint32_t ucs = c[2].z & 0xffffu;  // UDP checksum field (0: none, IPv4)
  const bool need_l4 = tcp || ucs != 0u;
  const int l4_len = tcp ? ip_paylen : (int)udp_len;
  const int E4 = 34 + l4_len;
  // IPv4 header words: window bytes [14, 34).
  const uint32_t s3 = chunk_sum_all(c[1], (c[0].w >> 16) + (c[2].x & 0xffffu));
  uint32_t reason = fold16(s3) != 0xffffu ? OO_RX_R_IP4_CSUM : PENDING;
  // Pseudo header (checksum.c:215-223) and the L4 words in the window [34, E4h).
  const uint32_t pseudo = (c[1].z >> 16) + (c[1].w & 0xffffu) + (c[1].w >> 16) + (c[2].x & 0xffffu) +
                          (tcp ? 0x0600u + bswap16((uint32_t)ip_paylen) : 0x1100u + (c[2].y >> 16));
  const int E4h = E4 > HB ? off0 : E4;  // the body stream covers [off0, ...)
  uint32_t s4 = 0;
  if (__ballot((E4h & 15) != 0) == 0) {  // the region ends on a cell edge (wave-uniform test)
#pragma unroll
    for (int k = 2; k < HC; ++k) {
      const uint32_t t = chunk_sum_all(c[k], 0u);
      s4 += E4h >= 16 * k + 16 ? t : 0u;
    }
    s4 -= E4h >= 48 ? (c[2].x & 0xffffu) : 0u;  // bytes 32-33: the IPv4 header's
  } else if (SPAN) {
    s4 = window_sum_cells<2>(W, c, 34, E4h);
  } else {
#pragma unroll
    for (int k = 2; k < HC; ++k)
      if (16 * k < E4h) s4 += chunk_sum(c[k], 16 * k, 34, E4h);
  }
  const bool longl4 = reason == PENDING && need_l4 && E4 > HB;
  if (reason == PENDING && need_l4 && !longl4 && fold16(fold16(s4) + pseudo) != 0xffffu)
    reason = tcp ? OO_RX_R_TCP_CSUM : OO_RX_R_UDP_CSUM;
  h.reason = reason;
  h.late = (tcp && frag != 0x4000u && frag != 0u) ? OO_RX_R_TCP_SCATTERED : PENDING;
  // The TCP timestamp-option fast layout (tcp_rx.c:4537-4543): bytes 46, 54-57.
  h.flags = (reason == PENDING && tcp && ((c[2].w >> 16) & 0xffu) == 0x80u &&
             ((c[3].y >> 16) | (c[3].z << 16)) == 0x0a080101u) ? OO_RX_F_TSO : 0u;
  h.vlan = 0;
  h.proto = proto;
  h.ip_paylen = (uint32_t)ip_paylen;
  h.l4 = 34;
  h.l3ok = true;
  h.is6 = false;
  h.longl4 = longl4;
  h.sport = c[2].x >> 16;
  h.dport = c[2].y & 0xffffu;
  h.sa[0] = (c[1].z >> 16) | (c[1].w << 16);
  h.da[0] = (c[1].w >> 16) | (c[2].x << 16);
#pragma unroll
  for (int i = 1; i < 4; ++i) h.sa[i] = h.da[i] = 0;
  h.s4 = s4;
  h.pseudo = need_l4 ? pseudo : 0u;
  h.E4 = need_l4 ? E4 : 34;
  return true;
}

// The fixed-format IPv6 header: 16-B-aligned start, untagged Ethernet, IPv6
// with TCP or UDP as the next header (netif_event.c:1060-1076: no extension
// header walk) whose length fields pass the gates.  L3 at window byte 14,
// addresses at 22 and 38, L4 at 54.  The same decisions as parse_general for
// these frames; false (h untouched) for every other frame.
template <bool SPAN>
__device__ __forceinline__ bool parse_fixed6(const Win& W, const uint4 (&c)[HC], int shift, int len,
                                             int off0, Hdr& h) {
  const int ip_paylen = (int)bswap16(c[1].x >> 16);
  const uint32_t proto = c[1].y & 0xffu;
  const uint32_t udp_len = bswap16(c[3].z >> 16);
  const int hlen = (int)(((c[4].x >> 16) & 0xf0u) >> 2);
  const bool tcp = proto == 6u;
  const bool ok = (shift == 0) & (off0 >= 64) & ((c[0].w & 0xffffu) == 0xdd86u) & (ip_paylen > 0) &
                  (len >= 54 + ip_paylen) &
                  (tcp ? ((ip_paylen >= 20) & (hlen >= 20) & (ip_paylen >= hlen))
                       : ((proto == 17u) & (ip_paylen >= 8) & (udp_len >= 8u) &
                          (udp_len <= (uint32_t)ip_paylen)));
  if (!ok) return false;
  const int E4 = 54 + (tcp ? ip_paylen : (int)udp_len);
  // Pseudo header (checksum.c:215-223): the 16 address words [22, 54), then
  // payload_len (TCP) or the UDP length field, and the protocol.
  uint32_t pseudo = (c[1].y >> 16) + (c[1].z & 0xffffu) + (c[1].z >> 16) + (c[1].w & 0xffffu) +
                    (c[1].w >> 16) + (c[3].x & 0xffffu) + (c[3].x >> 16) + (c[3].y & 0xffffu);
  pseudo = chunk_sum_all(c[2], pseudo) +
           (tcp ? (c[1].x >> 16) + 0x0600u : (c[3].z >> 16) + 0x1100u);
  // The L4 words in the window, [54, E4h).
  const int E4h = E4 > HB ? off0 : E4;
  uint32_t s4 = 0;
  if (__ballot((E4h & 15) != 0) == 0) {  // the region ends on a cell edge (wave-uniform test)
#pragma unroll
    for (int k = 3; k < HC; ++k) {
      const uint32_t t = chunk_sum_all(c[k], 0u);
      s4 += E4h >= 16 * k + 16 ? t : 0u;
    }
    s4 -= E4h >= 64 ? (c[3].x & 0xffffu) + (c[3].x >> 16) + (c[3].y & 0xffffu) : 0u;  // [48, 54)
  } else if (SPAN) {
    s4 = window_sum_cells<3>(W, c, 54, E4h);
  } else {
#pragma unroll
    for (int k = 3; k < HC; ++k)
      if (16 * k < E4h) s4 += chunk_sum(c[k], 16 * k, 54, E4h);
  }
  const bool longl4 = E4 > HB;
  h.reason = (!longl4 && fold16(fold16(s4) + pseudo) != 0xffffu)
                 ? (tcp ? OO_RX_R_TCP_CSUM : OO_RX_R_UDP_CSUM) : PENDING;
  h.late = PENDING;
  // The TCP timestamp-option fast layout (tcp_rx.c:4537-4543): bytes 66, 74-77.
  h.flags = OO_RX_F_IP6 |
            ((h.reason == PENDING && tcp && ((c[4].x >> 16) & 0xffu) == 0x80u &&
              ((c[4].z >> 16) | (c[4].w << 16)) == 0x0a080101u) ? OO_RX_F_TSO : 0u);
  h.vlan = 0;
  h.proto = proto;
  h.ip_paylen = (uint32_t)ip_paylen;
  h.l4 = 54;
  h.l3ok = true;
  h.is6 = true;
  h.longl4 = longl4;
  h.sport = c[3].y >> 16;
  h.dport = c[3].z & 0xffffu;
  h.sa[0] = (c[1].y >> 16) | (c[1].z << 16);
  h.sa[1] = (c[1].z >> 16) | (c[1].w << 16);
  h.sa[2] = (c[1].w >> 16) | (c[2].x << 16);
  h.sa[3] = (c[2].x >> 16) | (c[2].y << 16);
  h.da[0] = (c[2].y >> 16) | (c[2].z << 16);
  h.da[1] = (c[2].z >> 16) | (c[2].w << 16);
  h.da[2] = (c[2].w >> 16) | (c[3].x << 16);
  h.da[3] = (c[3].x >> 16) | (c[3].y << 16);
  h.s4 = s4;
  h.pseudo = pseudo;
  h.E4 = E4;
  return true;
}

// The header stage of one packet (one lane): the fixed-format paths when
// they apply, the general walk otherwise (handle_rx_csum_bad's gates and
// checksums, handle_rx_pkt's IPv4 checks).
// RUNS: the general walk by word runs (win_kernel; rx_kernel, at its
// register limit with the body ring's cursors live, keeps the byte walk).
template <bool RUNS>
__device__ __forceinline__ Hdr parse_headers(const Win& W, int shift, int len, uint64_t abase) {
  const int off0 = (int)body_off0(abase);
  Hdr h;
  bool fixed;
  {
    uint4 c[HC];
    read_cells(W, c);
    fixed = parse_fixed<RUNS && OO_RX_FIXED_SPAN>(W, c, shift, len, off0, h);
    DSTAMP(13);
    if (__ballot(!fixed && (c[0].w & 0xffffu) == 0xdd86u) != 0) {
      bool f6 = false;
      if (!fixed) f6 = parse_fixed6<RUNS && OO_RX_FIXED_SPAN>(W, c, shift, len, off0, h);
      fixed = fixed || f6;
    }
  }
  DSTAMP(14);
  if (__ballot(!fixed) != 0) {
    if (!fixed) h = RUNS ? parse_general_runs(W, shift, len, off0) : parse_general(W, shift, len, off0);
  }
  DSTAMP(15);
  return h;
}

// The 2 (UDP) or 3 (TCP) lookup stages of one lane in reference order; the
// first stage with a match decides (*stage = 1..3).  M as rec_match_m: a wave
// holding both families walks them together (M = 2), so its walks cost the
// dependent loads of one family, not of both in turn.
template <int M, bool PRE1, class PR>
__device__ __forceinline__ Match lookup_stages(const KParams& P, const PR& t, bool any6,
                                               const Hdr& h, uint32_t dport, uint32_t sport,
                                               uint32_t proto, uint32_t hwp, int vlan, bool tcp,
                                               uint32_t h1_0, uint32_t h1_1, uint32_t h1_2,
                                               bool o0, bool o1, bool o2, bool q0, bool q1,
                                               bool q2, Rec rec, int fs, int& stage,
                                               bool& s2) {
  const uint32_t zero[4] = {0, 0, 0, 0};
  const bool six = M == 1 || (M == 2 && t.is6);
  const uint32_t dx = six ? (h.da[0] ^ h.da[1] ^ h.da[2] ^ h.da[3]) : h.da[0];
  const uint32_t sx = six ? (h.sa[0] ^ h.sa[1] ^ h.sa[2] ^ h.sa[3]) : h.sa[0];
  // Stage 2's first record, when stage 1 did not get the up-front one, is
  // loaded beside stage 1's walk (ready when that walk ends without a match,
  // instead of one more dependent load after it).  PRE1: IPv4-only waves --
  // a second 64-B record in a wave holding IPv6 spills.
  Rec rec1 = rec;
  const bool pre1 = PRE1 && fs == 0 && o1;
  if (pre1) rec1 = load_rec(P, t, h1_1, any6);
  Match m = walk<M>(P, t, any6, h.da, dport, h.sa, false, sport, proto, hwp, vlan, h1_0,
                      hash2(dx, dport, sx, sport, proto), o0, rec, fs == 0, q0, tcp);
  DSTAMP(11);
  stage = 1;
  // Stage 2 for the lanes stage 1 left undecided and, for the future rule's
  // union (udp_internal.h:41-52, :86-97), for IPv4 UDP lanes with one
  // stage-1 match: there only whether it matches at all (OO_RX_F_UDP_S2).
  const bool probe = !tcp && !six && m.n == 1;
  s2 = false;
  if (m.n == 0 || probe) {
    const Match m2 = walk<M>(P, t, any6, h.da, dport, zero, true, 0u, proto, hwp, vlan, h1_1,
                             hash2(dx, dport, 0u, 0u, proto), o1, rec1, fs == 1 || pre1, q1,
                             tcp || probe);
    if (probe) {
      s2 = m2.n != 0;
    } else {
      m = m2;
      stage = 2;
    }
  }
  DSTAMP(12);
  if (m.n == 0 && tcp) {
    m = walk<M>(P, t, any6, zero, dport, zero, true, 0u, proto, hwp, vlan, h1_2,
                  hash2(0u, dport, 0u, 0u, proto), o2, rec, fs == 2, q2, true);
    stage = 3;
  }
  return m;
}

// The same lookups as one per-lane state machine (OO_RX_FSM): every step
// each live lane evaluates the slot whose record it holds, advances along
// its stage's probe sequence or on to its next stage (stages whose first
// slot is EMPTY, and a second slot known EMPTY, are passed without a load),
// and loads the next record it needs -- one dependent load per step for the
// whole wave.  The sequential walks cost a wave the sum over stages of its
// longest walk in each; this costs the longest per-lane total (config 5:
// 7.5 against 4.6 slot visits per 64 packets, tools/walk_levels.py).
#ifndef OO_RX_FSM
#define OO_RX_FSM 1
#endif
#ifndef OO_RX_FSM2
#define OO_RX_FSM2 1  // win_kernel: two slots per load level (lookup_fsm2)
#endif
template <int M, class PR>
__device__ __forceinline__ Match lookup_fsm(const KParams& P, const PR& t, bool any6,
                                            const Hdr& h, uint32_t dport, uint32_t sport,
                                            uint32_t proto, uint32_t hwp, int vlan, bool tcp,
                                            uint32_t h1_0, uint32_t h1_1, uint32_t h1_2,
                                            uint32_t h2_0, uint32_t h2_1, uint32_t h2_2, bool o0,
                                            bool o1, bool o2, bool q0, bool q1, bool q2, Rec rec,
                                            int fs, int& stage, bool& s2) {
  const uint32_t nst = tcp ? 3u : 2u;  // o2 (and q2) are false for UDP
  const bool six = M == 1 || (M == 2 && t.is6);
  (void)o0;
  Match m = {-1, 0};
  // probe: an IPv4 UDP lane decided in stage 1 with one match walks stage 2
  // for the future rule's union (udp_internal.h:41-52, :86-97): s2 = it
  // matches too.
  bool probe = false;
  s2 = false;
  uint32_t s = (uint32_t)fs;  // the first stage whose first slot is occupied (3: none)
  bool live = s < nst;
  uint32_t h1 = s == 0 ? h1_0 : s == 1 ? h1_1 : h1_2;
  uint32_t first = h1;
  uint32_t h2 = s == 0 ? h2_0 : s == 1 ? h2_1 : h2_2;
  uint32_t k = 0;    // probe index within the stage
  bool occ = true;   // slot h1 not EMPTY (rec is its record)
  uint32_t guard = 0;
  for (; __ballot(live) != 0 && guard <= 3u * (t.mask + 1u); ++guard) {
    if (live) {
      // The slot in hand (netif_table.c:192-231 / netif_table_ip6.c:146-170).
      bool end = !occ;  // an EMPTY slot ends the stage's walk
      if (occ) {
        const bool st0 = s == 0;
        uint32_t la[4], ra[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          la[i] = s < 2 ? h.da[i] : 0u;
          ra[i] = st0 ? h.sa[i] : 0u;
        }
        int32_t id;
        if (rec_match_m<M>(P, t, rec, k == 0, la, dport, ra, !st0, st0 ? sport : 0u, proto,
                           hwp, vlan, id)) {
          if (probe) {
            s2 = true;
            end = true;
          } else {
            if (m.n == 0) m.first = id;
            ++m.n;
            end = tcp;  // TCP's deliver callbacks end the walk at the first match
          }
        }
        if (!end) {
          h1 = (h1 + h2) & t.mask;
          end = h1 == first;  // a full cycle
          ++k;
          // the second slot's bit came with the first batch
          if (!end && k == 1) end = !(s == 0 ? q0 : s == 1 ? q1 : q2);
        }
      }
      if (end) {
        if (probe) {
          live = false;
        } else if (m.n != 0) {
          stage = (int)s + 1;  // this stage decides
          live = false;
          if (!tcp && !six && s == 0 && m.n == 1 && o1) {
            probe = true;  // and stage 2 is walked for the future rule
            live = true;
            s = 1;
            h1 = h1_1;
            first = h1;
            h2 = h2_1;
            k = 0;
          }
        } else {
          // on to the next stage whose first slot is occupied
          ++s;
          if (s == 1 && !o1) ++s;
          if (s == 2 && !o2) ++s;
          live = s < nst;
          h1 = s == 1 ? h1_1 : h1_2;
          first = h1;
          h2 = s == 1 ? h2_1 : h2_2;
          k = 0;
        }
      }
      // The next record (and, past the second slot, its occupancy bit with
      // it: an EMPTY slot's record is simply not used).
      if (live) {
        rec = load_rec(P, t, h1, any6);
        occ = k < 2 ? true : probe_occ(P, t, h1);
      }
    }
  }
  DSTAMPV(11, 1000000u + guard);  // the wave's steps (marked: not a time)
  return m;
}

// The state machine with the occupancy bits in LDS (win_kernel): every
// step also loads the record of the next slot on the lane's probe sequence
// when that slot is occupied, and evaluates it in the same step when the
// walk goes on to it -- two slots per dependent load along a chain (config
// 5's connected-socket chains).  The same walks,
// matches and stages as lookup_fsm; EMPTY slots are known from LDS before
// any load, so no record of an EMPTY slot is loaded.
template <int M>
__device__ __forceinline__ Match lookup_fsm2(const KParams& P, const ProbeL& t, bool any6,
                                             const Hdr& h, uint32_t dport, uint32_t sport,
                                             uint32_t proto, uint32_t hwp, int vlan, bool tcp,
                                             uint32_t h1_0, uint32_t h1_1, uint32_t h1_2,
                                             uint32_t h2_0, uint32_t h2_1, uint32_t h2_2, bool o1,
                                             bool o2, Rec rec, int fs, int& stage, bool& s2) {
  const uint32_t nst = tcp ? 3u : 2u;  // o2 is false for UDP
  const bool six = M == 1 || (M == 2 && t.is6);
  Match m = {-1, 0};
  bool probe = false;
  s2 = false;
  uint32_t s = (uint32_t)fs;
  bool live = s < nst;
  uint32_t h1 = s == 0 ? h1_0 : s == 1 ? h1_1 : h1_2;
  uint32_t first = h1;
  uint32_t h2 = s == 0 ? h2_0 : s == 1 ? h2_1 : h2_2;
  uint32_t k = 0;
  bool occ = true;  // slot h1 not EMPTY (rec is its record)
  // The second record: slot (h1 + h2) & mask, when it is occupied and not
  // the cycle's start.
  Rec rec2 = {};
  bool have2 = false;
  {
    const uint32_t n = (h1 + h2) & t.mask;
    have2 = live && n != first && probe_occ(P, t, n);
    if (have2) rec2 = load_rec(P, t, n, any6);
  }
  for (uint32_t guard = 0; __ballot(live) != 0 && guard <= 3u * (t.mask + 1u); ++guard) {
    if (live) {
      bool end = !occ;  // an EMPTY slot ends the stage's walk
      // Up to two slots of the same walk: rec (slot h1), then rec2.
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const bool eval = e == 0 ? !end : (!end && have2);
        if (eval) {
          const bool st0 = s == 0;
          uint32_t la[4], ra[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            la[i] = s < 2 ? h.da[i] : 0u;
            ra[i] = st0 ? h.sa[i] : 0u;
          }
          int32_t id;
          if (rec_match_m<M>(P, t, e == 0 ? rec : rec2, k == 0, la, dport, ra, !st0,
                             st0 ? sport : 0u, proto, hwp, vlan, id)) {
            if (probe) {
              s2 = true;
              end = true;
            } else {
              if (m.n == 0) m.first = id;
              ++m.n;
              end = tcp;  // TCP's deliver callbacks end the walk at the first match
            }
          }
          if (!end) {
            h1 = (h1 + h2) & t.mask;
            end = h1 == first;  // a full cycle
            ++k;
            // the next slot: its record came with this batch, or it is
            // EMPTY (or, after the second record, not loaded yet)
            if (!end && !(e == 0 && have2)) end = !probe_occ(P, t, h1);
          }
        }
      }
      if (end) {
        if (probe) {
          live = false;
        } else if (m.n != 0) {
          stage = (int)s + 1;  // this stage decides
          live = false;
          if (!tcp && !six && s == 0 && m.n == 1 && o1) {
            probe = true;  // and stage 2 is walked for the future rule
            live = true;
            s = 1;
            h1 = h1_1;
            first = h1;
            h2 = h2_1;
            k = 0;
          }
        } else {
          ++s;
          if (s == 1 && !o1) ++s;
          if (s == 2 && !o2) ++s;
          live = s < nst;
          h1 = s == 1 ? h1_1 : h1_2;
          first = h1;
          h2 = s == 1 ? h2_1 : h2_2;
          k = 0;
        }
      }
      // The records of slot h1 and the one after it, occupied ones only
      // (after two slots, h1 may be occupied without its record: it is
      // loaded here).
      have2 = false;
      if (live) {
        occ = probe_occ(P, t, h1);
        if (occ) {
          rec = load_rec(P, t, h1, any6);
          const uint32_t n = (h1 + h2) & t.mask;
          have2 = n != first && probe_occ(P, t, n);
          if (have2) rec2 = load_rec(P, t, n, any6);
        }
      }
    }
  }
  return m;
}

// The lookups through the key index (oo_rx_device.h; DESIGN.md "The key
// index"): every stage's key of the lane in one load level -- a 32-B bucket
// (IPv4; 48 B, with the next bucket's first entry, in a wave that also holds
// IPv6 lanes) or the first 48 B of a 64-B entry (IPv6) per key -- and another
// level only for a key whose bucket was full.  The index's flag word comes with them (a scalar load: no vector
// wait of its own).  Returns true for a lane whose m / stage / s2 it set as
// the walks would have; false for a lane that must walk: an answer that
// depends on the packet's interface or VLAN (bind2dev), a UDP key with
// other than one match, or an index the last table change turned off.
// `issued` runs once, right after the first level's loads are issued and
// before any of them is waited for (window_loop stages its next tile there,
// so the two round trips overlap); it issues exactly kIssuedOps
// vector-memory operations (window_loop's stage: a descriptor line, HC
// window rows, the claim), or none (the default, [] {}).
constexpr int kIssuedOps = HC + 2;
template <bool ANY6, bool STAGE, class F>
__device__ __forceinline__ bool kx_lookup(const KParams& P, const Hdr& h, bool look, bool tcp,
                                          bool any_tcp, uint32_t dport, uint32_t sport,
                                          uint32_t proto, bool o0, bool o1, bool o2, Match& m,
                                          int& stage, bool& s2, F&& issued) {
  const bool six = ANY6 && h.is6;
  uint32_t la[4], sa[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    la[i] = i == 0 || six ? h.da[i] : 0u;
    sa[i] = i == 0 || six ? h.sa[i] : 0u;
  }
  const uint32_t p0 = dport | (sport << 16);
  const uint32_t pw0 = six ? proto : 0u, pw1 = six ? proto | 0x100u : 0u;
  uint32_t pos[3];
  pos[0] = kx_hash(la[0], la[1], la[2], la[3], sa[0], sa[1], sa[2], sa[3], p0, pw0);
  pos[1] = kx_hash(la[0], la[1], la[2], la[3], 0u, 0u, 0u, 0u, dport, pw1);
  pos[2] = kx_hash(0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, dport, pw1);
  const uint32_t pmask = six ? sreg(P.kx_ne6) - 1u : sreg(P.kx_nb4) - 1u;
#pragma unroll
  for (int k = 0; k < 3; ++k) pos[k] &= pmask;
  const uint64_t b4 = sreg64(P.kx4), b6 = sreg64(P.kx6);
  const uint64_t t4 = b4 + (uint64_t)(sreg(P.kx_nb4) + KX_PAD4) * 32u;
  const uint64_t base = six ? b6 : (tcp ? t4 : b4);
  const uint32_t shift = six ? 6u : 5u;
  const int nk = any_tcp ? 3 : 2;
  uint32_t okw;
  {
    const uint64_t fa = sreg64(P.kx_ok);
    asm volatile("s_load_dword %0, %1, 0x0" : "=s"(okw) : "s"(fa));
  }
  uint32_t val[3] = {0u, 0u, 0u};
  // Only keys whose first table slot is occupied: any other walk ends at
  // once without a match (its key is not in the index either).
  bool pend[3] = {look && o0, look && o1, look && tcp && o2};
  // One level: every pending key's bucket (entry) loaded, then compared.
  // (IPv6-capable waves hold 36 VGPRs of buckets: staging under them spills,
  // so they stage first and overlap nothing)
  constexpr bool OVERLAP = STAGE && !ANY6;
  if (!OVERLAP) issued();
  auto level = [&](bool first) __attribute__((always_inline)) {
    uint4 d[3][3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      if (k < nk) {
        // (a key not looked up reads the region's first bucket: one line
        // for the wave, no branch around the batch)
#ifdef OO_RX_BOUND_KXLINE  // (timing bound, wrong records: every lane loads one bucket)
        const uint64_t a = base;
#else
        const uint64_t a = base + ((uint64_t)(pend[k] ? pos[k] : 0u) << shift);
#endif
        if (OVERLAP && first) {
          d[k][0] = gload16_untracked(a);
#ifdef OO_RX_BOUND_KX1  // (timing bound, wrong records: the bucket's first entry only)
          d[k][1] = make_uint4(0u, 0u, 0u, 0u);
#else
          d[k][1] = gload16_untracked(a + 16u);
#endif
        } else {
          d[k][0] = gload16(a);
          d[k][1] = gload16(a + 16u);
          if (ANY6) d[k][2] = gload16(a + 32u);
        }
      }
    }
    if (OVERLAP && first) {
      // The loads are untracked: the compiler sees their values defined at
      // once, so neither its compares nor any wait of its own move above
      // `issued`; one counted wait after it covers them -- `issued` issues
      // exactly kIssuedOps vector-memory operations, all newer.
      issued();
      vm_wait<kIssuedOps>();
      // (the values as written by the loads, from here on)
#pragma unroll
      for (int k = 0; k < 3; ++k)
        if (k < nk)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            asm volatile("" : "+v"(d[k][j].x), "+v"(d[k][j].y), "+v"(d[k][j].z), "+v"(d[k][j].w));
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      if (k < nk && pend[k]) {
        const uint32_t kra = k == 0 ? sa[0] : 0u, kp = k == 0 ? p0 : dport;
        const uint32_t kla = k == 2 ? 0u : la[0];
        uint32_t hv = 0u;
        bool empty = false;
#pragma unroll
        for (int j = 0; j < (ANY6 ? 3 : 2); ++j) {
          const uint4 e = d[k][j];
          const bool hj = (e.w != 0u) & (e.x == kla) & (e.y == kra) & (e.z == kp);
          hv = hj ? e.w : hv;
          empty |= e.w == 0u;
        }
        if (ANY6 && six) {
          bool eq = (d[k][2].z != 0u) & (d[k][2].x == kp) & (d[k][2].y == (k == 0 ? pw0 : pw1));
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const uint32_t ei = i == 0 ? d[k][0].x : i == 1 ? d[k][0].y : i == 2 ? d[k][0].z : d[k][0].w;
            const uint32_t ri = i == 0 ? d[k][1].x : i == 1 ? d[k][1].y : i == 2 ? d[k][1].z : d[k][1].w;
            eq = eq & (ei == (k == 2 ? 0u : la[i])) & (ri == (k == 0 ? sa[i] : 0u));
          }
          hv = eq ? d[k][2].z : 0u;
          empty = d[k][2].z == 0u;
        }
        if (hv != 0u) {
          val[k] = hv;
          pend[k] = false;
        } else if (empty) {
          pend[k] = false;
        } else {
          pos[k] += 1u;
        }
      }
    }
  };
  // The first level is issued at once (a loop head would first wait for
  // every load in flight, the body stream's included); the loop takes the
  // rare keys whose bucket was full.
  DSTAMP(9);
  level(true);
  DSTAMP(10);
  bool left = false;
  for (uint32_t it = 1;; ++it) {
    const bool any = pend[0] || pend[1] || pend[2];
    if (__ballot(any) == 0) break;
    if (it > KX_OVF + 2u) {  // (cannot happen: a pad bucket is always empty)
      left = any;
      break;
    }
    level(false);
  }
  DSTAMP(11);
  asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(okw));
  const bool f0 = val[0] != 0u, f1 = val[1] != 0u, f2 = tcp && val[2] != 0u;
  bool fb = left;
  uint32_t v = 0u;
  if (f0) {
    v = val[0];
    stage = 1;
    if (!tcp && !six) {  // IPv4 UDP: stage 2 for the future rule (lookup_stages)
      s2 = f1;
      fb = fb || (f1 && (val[1] & KX_FB) != 0u);
    }
  } else if (f1) {
    v = val[1];
    stage = 2;
  } else if (f2) {
    v = val[2];
    stage = 3;
  }
  fb = fb || (v & KX_FB) != 0u || okw == 0u;
  m.first = v != 0u ? (int32_t)(v & ID_MASK) : -1;
  m.n = v != 0u ? 1u : 0u;
  return look && !fb;
}

// The record of one packet from its headers: the lookup stages of
// ci_udp_handle_rx (udp_rx.c:271-306: full 4-tuple, then (laddr, lport)) or
// ci_tcp_handle_rx (tcp_rx.c:4786-4835: then (*, lport)); the first stage
// with a match decides.  IPv4 and IPv6 lanes share one instruction stream:
// every stage's first-slot and next-slot occupancy bits are loaded together,
// then the first slots' records, so a wave pays two dependent loads however
// its packets mix address families and protocols.
// LO: the occupancy bitmaps and the hwport bytes are in LDS at lds_occ
// (OccLds layout, win_kernel).
// `issued` (window_loop's next-tile staging) runs exactly once: after the
// key index's first loads are issued, or -- no lane looking up, or the index
// off -- before any of the lookup's loads.
template <bool ANY6, bool LO, bool STAGE, class F>
__device__ __forceinline__ Parsed demux_packet_t(const KParams& P, const Hdr& h, int intf_i,
                                                 uint64_t abase, int span, int shift,
                                                 uint32_t lds_occ, F&& issued) {
  const int vlan = (int)h.vlan;
  const uint32_t proto = h.proto;
  uint32_t reason = h.reason;
  uint32_t flags = h.flags;
  const bool is6 = h.is6;

  // Lanes that reach the lookups.  The record is assembled after them: its
  // fields come from the headers, which the lookups hold anyway.
  const bool csum_ok = reason == PENDING;
#ifdef OO_RX_BOUND_NOLOOK  // (a timing bound, wrong records: no lookup at all)
  const bool look = false;
#else
  const bool look = csum_ok && h.late == PENDING;
#endif
  const uint32_t sport = h.sport, dport = h.dport;
  const uint32_t sx = is6 ? h.sa[0] ^ h.sa[1] ^ h.sa[2] ^ h.sa[3] : h.sa[0];  // hash addresses
  const uint32_t dx = is6 ? h.da[0] ^ h.da[1] ^ h.da[2] ^ h.da[3] : h.da[0];
  Match m = {-1, 0};
  int stage = 0;
  bool s2 = false;
  if (__ballot(look) != 0) {
    constexpr bool any6 = ANY6;
    typedef typename std::conditional<LO, ProbeL, Probe>::type PR;
    PR t;
    static_cast<Probe&>(t) = probe_of(P, ANY6 && is6);
    // (intf_i_to_hwport for a valid interface; lanes with none read entry 0
    // and take 0xff)
    const bool intf_ok = (uint32_t)intf_i < (uint32_t)OO_GPU_RX_MAX_INTF;
    uint64_t hwa;
    if constexpr (LO) {
      t.lo = lds_occ + (ANY6 && is6 ? OCC_LDS_B6 : 0u);
      hwa = lds_occ + OCC_LDS_HW + (intf_ok ? (uint32_t)intf_i : 0u);
    } else {
      hwa = sreg64(P.hwport) + (intf_ok ? (uint32_t)intf_i : 0u);
    }
    uint32_t hwp = 0xffu;
    const bool tcp = proto == 6u;
    const uint32_t h1_0 = hash3(dx, dport, sx, sport, proto) & t.mask;
    const uint32_t h1_1 = hash3(dx, dport, 0u, 0u, proto) & t.mask;
    const uint32_t h1_2 = hash3(0u, dport, 0u, 0u, proto) & t.mask;
    const uint32_t h2_0 = hash2(dx, dport, sx, sport, proto);
    const uint32_t h2_1 = hash2(dx, dport, 0u, 0u, proto);
    const uint32_t h2_2 = hash2(0u, dport, 0u, 0u, proto);
    // All the bits in one batch: six words, or four when no lane of the
    // wave looks up TCP (UDP has no third stage).
    bool o0 = false, o1 = false, o2 = false, q0 = false, q1 = false, q2 = false;
    const bool any_tcp = __ballot(look && tcp) != 0;
    if (look) {
      const uint32_t idx[6] = {h1_0, h1_1, h1_2, (h1_0 + h2_0) & t.mask, (h1_1 + h2_1) & t.mask,
                               (h1_2 + h2_2) & t.mask};
      uint32_t w[6], hw;
      if (any_tcp) {
        occ_words6(t, idx, w, hwa, hw);
      } else {
        const uint32_t i4[4] = {idx[0], idx[1], idx[3], idx[4]};
        uint32_t w4[4];
        occ_words4(t, i4, w4, hwa, hw);
        w[0] = w4[0];
        w[1] = w4[1];
        w[3] = w4[2];
        w[4] = w4[3];
        w[2] = w[5] = 0u;
      }
      DSTAMP(8);
      hwp = intf_ok ? (hw & 0xffu) : 0xffu;
      auto bit = [&](int k) { return ((w[k] >> (idx[k] & 31u)) & 1u) != 0; };
      o0 = bit(0);
      o1 = bit(1);
      o2 = bit(2) && tcp;
      q0 = bit(3);
      q1 = bit(4);
      q2 = bit(5) && tcp;
    }
    // One record per lane up front: the first slot of the first stage whose
    // first slot is occupied (a stage with an EMPTY first slot ends at once,
    // and that record usually decides); a later stage loads its own only
    // when this one did not match.
    const int fs = o0 ? 0 : o1 ? 1 : o2 ? 2 : 3;
    // Lanes that walk the tables: all that look up, less those the key
    // index answers.
    bool walkl = look;
    if (P.kx4 != nullptr) {
      // (every lane: `issued` needs the whole wave; a lane that does not
      // look up loads a dummy bucket and matches nothing)
      const bool kxa = kx_lookup<ANY6, STAGE>(P, h, look, tcp, any_tcp, dport, sport, proto, o0, o1, o2, m,
                                       stage, s2, issued);
      walkl = look && !kxa;
    } else {
      issued();
    }
    Rec rec = {};
    if (walkl && fs < 3) rec = load_rec(P, t, fs == 0 ? h1_0 : fs == 1 ? h1_1 : h1_2, any6);
    if (walkl) {
      DSTAMP(9);
      // Both families walk in one instruction stream (lookup_stages<2>).
      // Waves with TCP lookups (three stages, long connected-socket chains)
      // take the state machine; UDP-only waves the stage-by-stage walks.
      if constexpr (LO) {
        if (OO_RX_FSM2 && any_tcp)
          m = lookup_fsm2<ANY6 ? 2 : 0>(P, t, any6, h, dport, sport, proto, hwp, vlan, tcp, h1_0, h1_1,
                                        h1_2, h2_0, h2_1, h2_2, o1, o2, rec, fs, stage, s2);
        else if (OO_RX_FSM && any_tcp)
          m = lookup_fsm<ANY6 ? 2 : 0>(P, t, any6, h, dport, sport, proto, hwp, vlan, tcp, h1_0, h1_1,
                                       h1_2, h2_0, h2_1, h2_2, o0, o1, o2, q0, q1, q2, rec, fs, stage,
                                       s2);
        else
          m = lookup_stages<ANY6 ? 2 : 0, !ANY6>(P, t, any6, h, dport, sport, proto, hwp, vlan, tcp,
                                                 h1_0, h1_1, h1_2, o0, o1, o2, q0, q1, q2, rec, fs,
                                                 stage, s2);
      } else if (OO_RX_FSM && any_tcp)
        m = lookup_fsm<ANY6 ? 2 : 0>(P, t, any6, h, dport, sport, proto, hwp, vlan, tcp, h1_0, h1_1,
                                     h1_2, h2_0, h2_1, h2_2, o0, o1, o2, q0, q1, q2, rec, fs, stage,
                                     s2);
      else
        m = lookup_stages<ANY6 ? 2 : 0, !ANY6>(P, t, any6, h, dport, sport, proto, hwp, vlan, tcp,
                                               h1_0, h1_1, h1_2, o0, o1, o2, q0, q1, q2, rec, fs, stage,
                                               s2);
      DSTAMP(10);
    }
  } else {
    issued();
  }
  DSTAMP(12);
  oo_gpu_rx_result r;
  r.reason = 0; r.flags = 0; r.stage = 0; r.proto = 0; r.vlan = (uint16_t)vlan;
  r.l4_off = 0; r.ip_paylen = 0; r.sport_be = 0; r.dport_be = 0; r.nmatch = 0;
  r.saddr_be = 0; r.daddr_be = 0; r.sock = -1; r.hash3 = 0;
  if (h.l3ok) {
    r.proto = (uint8_t)proto;
    r.ip_paylen = (uint16_t)h.ip_paylen;
  }
  if (csum_ok) {
    flags |= OO_RX_F_CSUM_OK;
    r.l4_off = (uint16_t)h.l4;
    r.sport_be = (uint16_t)sport;
    r.dport_be = (uint16_t)dport;
    r.saddr_be = sx;
    r.daddr_be = dx;
    reason = h.late;
  }
  if (look) {
    r.hash3 = hash3(dx, dport, sx, sport, proto);
    if (proto == 17u) {
      // ci_udp_rx_deliver's multi-destination test reads the IPv4 view of
      // the L3 header (udp_rx.c:157-159): bytes 16..19, which for IPv6 are
      // source-address bytes 8..11.
      const uint32_t dd = is6 ? h.sa[2] : h.da[0];
      if ((dd & 0xf0u) == 0xe0u || dd == 0xffffffffu) flags |= OO_RX_F_MCAST;
    }
    reason = OO_RX_R_NO_MATCH;
    if (m.n) {
      reason = OO_RX_R_DELIVER;
      r.stage = (uint8_t)stage;
      r.sock = m.first;
      r.nmatch = (uint16_t)m.n;
      if (m.n > 1) flags |= OO_RX_F_MULTI;
      if (s2) flags |= OO_RX_F_UDP_S2;
    }
  }
  r.reason = (uint8_t)reason;
  r.flags = (uint8_t)flags;
  Parsed ps;
  ps.r = r;
  ps.s4 = h.s4;
  ps.pseudo = h.pseudo;
  // The body stream covers window bytes [off0, span); an L4 region that
  // ends before the frame does leaves its complement to subtract.
  if (h.longl4 && h.E4 < span) ps.s4 -= window_sum_global(abase, h.E4, span);
  ps.odd_long = (uint32_t)(shift & 1) | (h.longl4 ? 2u : 0u);
  return ps;
}

// A wave whose lookups are all IPv4 takes the IPv4-only instance (the
// IPv6 compares and record halves compiled out).
// STAGE: `issued` issues kIssuedOps operations (window_loop's staging);
// otherwise it issues none.
template <bool LO = false, bool STAGE = false, class F>
__device__ __forceinline__ Parsed demux_packet(const KParams& P, const Hdr& h, int intf_i,
                                               uint64_t abase, int span, int shift,
                                               uint32_t lds_occ, F&& issued) {
  if (__ballot(h.is6 && h.reason == PENDING && h.late == PENDING) != 0)
    return demux_packet_t<true, LO, STAGE>(P, h, intf_i, abase, span, shift, lds_occ, issued);
  return demux_packet_t<false, LO, STAGE>(P, h, intf_i, abase, span, shift, lds_occ, issued);
}
template <bool LO = false>
__device__ __forceinline__ Parsed demux_packet(const KParams& P, const Hdr& h, int intf_i,
                                               uint64_t abase, int span, int shift,
                                               uint32_t lds_occ = 0) {
  return demux_packet<LO, false>(P, h, intf_i, abase, span, shift, lds_occ, [] {});
}

// The verdict a long packet's record waited for: the window part plus the
// body; a failure turns the record into the drop record (only the fields a
// drop defines survive).
__device__ __forceinline__ void finish(Parsed& ps, uint32_t body) {
  if (!(ps.odd_long & 2u)) return;
  uint32_t f = fold16(ps.s4 + body);
  if (ps.odd_long & 1u) f = swap16(f);  // RFC 1071 byte-order swap
  if (fold16(f + ps.pseudo) != 0xffffu) {
    oo_gpu_rx_result& r = ps.r;
    r.reason = (uint8_t)(r.proto == 6u ? OO_RX_R_TCP_CSUM : OO_RX_R_UDP_CSUM);
    r.flags = (uint8_t)(r.flags & (OO_RX_F_VLAN | OO_RX_F_IP6));
    r.stage = 0; r.l4_off = 0; r.sport_be = 0; r.dport_be = 0; r.nmatch = 0;
    r.saddr_be = 0; r.daddr_be = 0; r.sock = -1; r.hash3 = 0;
  }
}

// ---------------------------------------------------------------------------
// Body streaming engine.
//
// A frame's body is its 16-B chunks from a0, the 128-B line holding window
// byte HB, to the frame end (the last chunk may be partial).  The parse covers
// the window bytes before a0.
//
// The tile's frames with a body are its jobs.  Job q goes to lane (g, j) =
// (q & 7, q >> 3); 8-lane group g streams its jobs j = 0, 1, ... one after
// the other, 8 x 16 B = one 128-B line per round, so one 1-KiB piece (one
// LDS-DMA instruction) is one round of all eight groups, and every round reads
// whole lines (a round straddling two lines reads HBM ~20 % slower:
// tools/ring_probe.hip).  All groups move to the next job slot on the same
// round: slot j lasts R_j rounds, the most any of its eight jobs needs.  When
// the tile's frames differ in size they are first ranked by size, so the jobs
// of a slot are alike.  Consuming a round is four dot products with a
// per-lane word weight (0 for lanes past their job's end); a job's partial
// last chunk takes a masked sum in the round that holds it.  The job/slot
// bookkeeping is scalar.

struct Jobs {       // a tile's jobs: lane (g, j) holds job q = g + 8 j
  uint32_t lo, hi;  // a0
  uint32_t nb;      // chunks from a0 (0: no job)
  uint32_t lim;     // frame end relative to a0
  uint32_t rj;      // R_(lane & 7): rounds of that job slot
  uint32_t T;       // rounds of the tile
};

// max(v) over lanes lane ^ 8, lane ^ 16 and lane ^ 32 (the lanes with the
// same lane & 7) -- DPP, swizzle and permlane32_swap: no address VGPRs (a
// per-lane bpermute address is a loop-invariant VGPR the kernel would spill).
__device__ __forceinline__ uint32_t max_x8(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, false));  // row_ror:8
  v = max(v, (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x401f));  // lane ^ 16
  const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);  // lane ^ 32
  return max((uint32_t)p[0], (uint32_t)p[1]);
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v, uint32_t lane) {
  (void)lane;
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xb1, 0xf, 0xf, false));   // [1,0,3,2]
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4e, 0xf, 0xf, false));   // [2,3,0,1]
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xf, 0xf, false));  // half mirror
  v = max_x8(v);
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

// Rank of each lane's key among the wave's, largest first, ties in lane
// order (a stable LSD radix sort on ballots; `bits` wave-uniform).
__device__ __forceinline__ uint32_t rank_desc(uint32_t key, uint32_t lane, int bits) {
  uint32_t k = key, id = lane;  // position `lane` holds (k, id)
  for (int b = 0; b < bits; ++b) {
    const bool one = (k >> b) & 1u;
    const uint64_t ones = __ballot(one);
    const uint32_t n1 = (uint32_t)__popcll(ones);
    const uint32_t o_below = __builtin_amdgcn_mbcnt_hi(
        (uint32_t)(ones >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ones, 0u));
    const uint32_t dst = one ? o_below : n1 + lane - o_below;
    k = (uint32_t)__builtin_amdgcn_ds_permute((int)(dst << 2), (int)k);
    id = (uint32_t)__builtin_amdgcn_ds_permute((int)(dst << 2), (int)id);
  }
  return (uint32_t)__builtin_amdgcn_ds_permute((int)(id << 2), (int)lane);  // to lane id: its rank
}

// The jobs of the tile whose lanes hold (abase, span); myslot = the lane that
// will hold this lane's body sum.  All lanes active.
__device__ __forceinline__ Jobs jobs_setup(uint64_t abase, int span, uint32_t lane,
                                           uint32_t& myslot) {
  const uint32_t off0 = body_off0(abase);
  const uint32_t nb = body_chunks(off0, span);
  const uint32_t rounds = (nb + 7u) >> 3;
  const uint64_t bm = __ballot(nb != 0);
  if (bm == 0) {  // no frame reaches past its window (64-B frames): no jobs
    myslot = lane;
    Jobs J;
    J.lo = J.hi = J.nb = J.lim = J.rj = J.T = 0;
    return J;
  }
  uint32_t myq;
  const uint32_t r0 = bm ? (uint32_t)__builtin_amdgcn_readlane((int)rounds, __builtin_ctzll(bm)) : 0u;
  const bool alike = __ballot(nb != 0 && rounds != r0) == 0;
  if (alike) {  // all jobs alike: list order
    const uint32_t M = (uint32_t)__popcll(bm);
    const uint32_t below = __builtin_amdgcn_mbcnt_hi(
        (uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
    myq = nb != 0 ? below : M + lane - below;  // a permutation of 0..63
  } else {
    myq = rank_desc(rounds, lane, 32 - __builtin_clz(wave_max(rounds, lane)));
  }
#if OO_RX_GSEQ
  // Job q (by size, largest first) goes to group g at position p = q / 8:
  // every group holds eight jobs, one from each pass of eight.
  {
    const uint32_t p = myq >> 3, i = myq & 7u;
    // snake order (0..7, 7..0, ...): the groups' round totals come out alike
    myslot = ((p & 1u) ? 7u - i : i) * 8u + p;
  }
#else
  myslot = (myq & 7u) * 8u + (myq >> 3);
#endif
  const uint32_t jp = (uint32_t)__builtin_amdgcn_ds_permute((int)(myslot << 2), (int)lane);
  const uint64_t a0 = abase + off0;
  Jobs J;
  J.lo = lane_get((uint32_t)a0, jp);
  J.hi = lane_get((uint32_t)(a0 >> 32), jp);
  J.nb = lane_get(nb, jp);
  J.lim = lane_get((uint32_t)span - off0, jp);
#if OO_RX_GSEQ
  // this lane's job's rounds; the tile takes the longest group's total
  J.rj = (J.nb + 7u) >> 3;
  J.T = wave_max(group_sum8(J.rj), lane);
#else
  // R_j: the most rounds over lanes 8g + j
  J.rj = max_x8((J.nb + 7u) >> 3);
  J.T = (uint32_t)__builtin_amdgcn_readlane((int)group_sum8(J.rj), 0);
#endif
  return J;
}

#if OO_RX_GSEQ
// Per-group job sequences (OO_RX_GSEQ): each 8-lane group streams its eight
// jobs back to back and moves to its next job on its own round, so a round
// carries every group's line until the group's sequence ends (lockstep job
// slots wait for the slot's longest job: config 4 carries 142 rounds of
// lines per tile for 111 rounds of bytes).  The cursors are per lane (one
// value per group); a group past its last job reads the zero line.
constexpr uint32_t NOJOB = 0xffffffffu;  // "no job": a round never reached

// Rounds are counted per cursor in k, wave-uniform (one scalar add a round);
// each lane keeps the rounds at which its group's job ends and after which
// its own chunk stops advancing as absolute counts, so a round costs one
// vector compare more than the lockstep slots.
struct IssueCursor {
  uint32_t k;       // rounds issued (wave-uniform)
  uint32_t js;      // the group's job position
  uint32_t kend;    // k at which the group's job ends (NOJOB: none)
  uint32_t kadv;    // k after which a stops advancing
  uint64_t a;       // the chunk this lane reads next
};

// Point the cursor at position js of the lane's group, at round k.  A lane
// past its job's last chunk keeps reading that chunk (a line of the same
// job); a group with no job there reads the zero line.  All lanes active.
__device__ __forceinline__ void issue_job(IssueCursor& c, const Jobs& J, uint32_t js,
                                          uint32_t lane, uint64_t zero) {
  const uint32_t gj = lane & 7u, s = (lane & ~7u) + min(js, 7u);
  const uint32_t nb0 = lane_get(J.nb, s), lo = lane_get(J.lo, s), hi = lane_get(J.hi, s);
  const uint32_t nb = js < 8u ? nb0 : 0u;
  const bool own = nb > gj;
  c.js = js;
  c.kend = nb != 0 ? c.k + ((nb + 7u) >> 3) : NOJOB;
  c.kadv = c.k + (own ? (nb - gj - 1u) >> 3 : 0u);
  const uint64_t a0 = (uint64_t)hi << 32 | lo;
  c.a = nb == 0 ? zero : a0 + (own ? gj : nb - 1u) * 16u;
}

__device__ __forceinline__ void issue_slot(IssueCursor& c, const Jobs& J, uint32_t js,
                                           uint32_t lane, uint64_t zero) {
  c.k = 0;
  issue_job(c, J, js, lane, zero);
}

// Issues the cursor's round into `slot`; groups whose job ends move on.
__device__ __forceinline__ void issue_round(IssueCursor& c, const Jobs& J, uint64_t zero,
                                            void* slot, uint32_t lane) {
  glds<OO_RX_BODY_AUX>(c.a, slot);
  c.a += c.k < c.kadv ? 128u : 0u;
  ++c.k;
  const bool sw = c.k == c.kend;
  if (__ballot(sw) != 0) {  // some group's job ends
    IssueCursor n;
    n.k = c.k;
    issue_job(n, J, c.js + 1u, lane, zero);
    if (sw) {
      c.js = n.js;
      c.kend = n.kend;
      c.kadv = n.kadv;
      c.a = n.a;
    }
  }
}

struct ConsumeCursor {
  uint32_t k;           // rounds consumed (wave-uniform)
  uint32_t js, kend;    // per group, as IssueCursor
  uint32_t klv;         // k up to which this lane has chunks of the job
  uint32_t vb;          // bytes of its last chunk in the frame (1..16)
  uint4 m;              // byte mask of its last chunk
  uint32_t acc;         // this lane's running sum
  uint32_t bs;          // the total of job (group, lane & 7); 0 if none
};

// mtab: an LDS table of the 17 byte masks by valid-byte count (body_kernel),
// or nullptr: computed.
__device__ __forceinline__ void consume_job(ConsumeCursor& c, const Jobs& J, uint32_t js,
                                            uint32_t lane, const uint4* mtab = nullptr) {
  const uint32_t gj = lane & 7u, s = (lane & ~7u) + min(js, 7u);
  const uint32_t nb0 = lane_get(J.nb, s), lim = lane_get(J.lim, s);
  const uint32_t nb = js < 8u ? nb0 : 0u;
  const uint32_t lv = nb > gj ? (nb - gj + 7u) >> 3 : 0u;  // rounds with a chunk
  c.js = js;
  c.kend = nb != 0 ? c.k + ((nb + 7u) >> 3) : NOJOB;
  c.klv = c.k + lv;
  const int last = 16 * (int)(gj + 8u * (lv - 1u));  // this lane's last chunk
  c.vb = (uint32_t)min(max((int)lim - last, 0), 16);
  if (mtab != nullptr) {
    c.m = lds_read16(&mtab[c.vb]);
  } else {
    auto bytes = [](int k) -> uint32_t {
      return k >= 4 ? 0xffffffffu : k <= 0 ? 0u : (1u << (8 * k)) - 1u;
    };
    const int vb = (int)c.vb;
    c.m = make_uint4(bytes(vb), bytes(vb - 4), bytes(vb - 8), bytes(vb - 12));
  }
}

__device__ __forceinline__ void consume_start(ConsumeCursor& c, const Jobs& J, uint32_t lane,
                                              const uint4* mtab = nullptr) {
  c.k = 0;
  consume_job(c, J, 0, lane, mtab);
  c.acc = 0;
  c.bs = 0;
}

// Consumes one round from the landed bytes v (lanes past their chunks weigh
// their words by 0); a group whose job ends folds its eight lane sums into
// the job's lane and moves on.
__device__ __forceinline__ void consume_round(ConsumeCursor& c, const Jobs& J, const uint4& v,
                                              uint32_t lane, const uint4* mtab = nullptr) {
  const bool live = c.k < c.klv;
  const bool part = live && c.k + 1u == c.klv && c.vb != 16u;
  if (__ballot(part) == 0) {
    const uint32_t w = live ? 0x00010001u : 0u;
    uint32_t a = dot(v.x, w, c.acc);
    uint32_t b = dot(v.y, w, 0u);
    a = dot(v.z, w, a);
    b = dot(v.w, w, b);
    c.acc = a + b;
  } else {  // some lane holds a frame's partial last chunk: byte masks
    const uint32_t f = live ? 0xffffffffu : 0u;
    const uint4 mm = part ? c.m : make_uint4(f, f, f, f);
    uint32_t a = dot(v.x & mm.x, 0x00010001u, c.acc);
    uint32_t b = dot(v.y & mm.y, 0x00010001u, 0u);
    a = dot(v.z & mm.z, 0x00010001u, a);
    b = dot(v.w & mm.w, 0x00010001u, b);
    c.acc = a + b;
  }
  ++c.k;
  const bool end = c.k == c.kend;
  if (__ballot(end) != 0) {  // some group's job ends
    const uint32_t t = group_sum8(c.acc);
    ConsumeCursor n;
    n.k = c.k;
    consume_job(n, J, c.js + 1u, lane, mtab);
    if (end) {
      if ((lane & 7u) == c.js) c.bs = t;
      c.acc = 0;
      c.js = n.js;
      c.kend = n.kend;
      c.klv = n.klv;
      c.vb = n.vb;
      c.m = n.m;
    }
  }
}
#else
__device__ __forceinline__ uint32_t slot_rounds(const Jobs& J, uint32_t js) {
  return js < 8u ? (uint32_t)__builtin_amdgcn_readlane((int)J.rj, (int)js) : 0u;
}

struct IssueCursor {
  uint32_t js, rnd, R;  // job slot, round in it, its rounds (wave-uniform)
  uint32_t adv;         // rounds after which a stops advancing
  uint64_t a;           // the chunk this lane reads next
};

// Point the issue cursor at job slot js (R = 0: past the last).  A lane past
// its job's end keeps reading the job's last chunk it read; a lane whose
// group has no job in the slot reads what the same lane of group 0 reads
// (group 0 has a job in every slot that is not past the last): the same
// lines as the instruction's live lanes, so no extra HBM traffic, and the
// consume side masks them.  Only a slot whose group-0 job is shorter than
// eight chunks leaves lanes on the zero line.  All lanes active.
__device__ __forceinline__ void issue_slot(IssueCursor& c, const Jobs& J, uint32_t js,
                                           uint32_t lane, uint64_t zero) {
  const uint32_t gj = lane & 7u, jj = min(js, 7u), s = (lane & ~7u) + jj;
  const uint32_t nb = lane_get(J.nb, s), lo = lane_get(J.lo, s), hi = lane_get(J.hi, s);
  const uint32_t nb0 = lane_get(J.nb, jj), lo0 = lane_get(J.lo, jj), hi0 = lane_get(J.hi, jj);
  c.js = js;
  c.rnd = 0;
  c.R = slot_rounds(J, js);
  const bool own = nb > gj, g0 = nb == 0 && nb0 > gj;
  const uint32_t n = own ? nb : nb0;
  c.adv = (own || g0) ? (n - gj - 1u) >> 3 : 0u;
  c.a = c.R == 0 ? zero
        : own   ? ((uint64_t)hi << 32 | lo) + gj * 16u
        : g0    ? ((uint64_t)hi0 << 32 | lo0) + gj * 16u
        : nb != 0 ? ((uint64_t)hi << 32 | lo) + (nb - 1u) * 16u
                  : zero;
}

// Issues the cursor's round into `slot`.
__device__ __forceinline__ void issue_round(IssueCursor& c, const Jobs& J, uint64_t zero,
                                            void* slot, uint32_t lane) {
  glds<OO_RX_BODY_AUX>(c.a, slot);
  c.a += c.rnd < c.adv ? 128u : 0u;
  if (++c.rnd == c.R) issue_slot(c, J, c.js + 1, lane, zero);
}

struct ConsumeCursor {
  uint32_t js, rnd, R;  // wave-uniform
  uint32_t lv;          // rounds of the slot in which this lane has a chunk
  uint32_t vb;          // bytes of its last chunk in the frame (1..16)
  uint4 m;              // byte mask of its last chunk
  uint32_t acc;         // this lane's running sum
  uint32_t bs;          // the total of job (group, lane & 7); 0 if none
};

__device__ __forceinline__ void consume_slot(ConsumeCursor& c, const Jobs& J, uint32_t js,
                                             uint32_t lane) {
  const uint32_t gj = lane & 7u, s = (lane & ~7u) + min(js, 7u);
  const uint32_t nb = lane_get(J.nb, s), lim = lane_get(J.lim, s);
  c.js = js;
  c.rnd = 0;
  c.R = slot_rounds(J, js);
  c.lv = (c.R != 0 && nb > gj) ? (nb - gj + 7u) >> 3 : 0u;
  const int last = 16 * (int)(gj + 8u * (c.lv - 1u));  // this lane's last chunk
  c.vb = (uint32_t)min(max((int)lim - last, 0), 16);
  auto bytes = [](int k) -> uint32_t {
    return k >= 4 ? 0xffffffffu : k <= 0 ? 0u : (1u << (8 * k)) - 1u;
  };
  const int vb = (int)c.vb;
  c.m = make_uint4(bytes(vb), bytes(vb - 4), bytes(vb - 8), bytes(vb - 12));
}

__device__ __forceinline__ void consume_start(ConsumeCursor& c, const Jobs& J, uint32_t lane) {
  consume_slot(c, J, 0, lane);
  c.acc = 0;
  c.bs = 0;
}

// Consumes one round from the landed bytes v (lanes past their chunks weigh
// their words by 0).
__device__ __forceinline__ void consume_round(ConsumeCursor& c, const Jobs& J, const uint4& v,
                                              uint32_t lane) {
  const bool live = c.rnd < c.lv;
  const bool part = live && c.rnd + 1u == c.lv && c.vb != 16u;
  if (__ballot(part) == 0) {
    const uint32_t w = live ? 0x00010001u : 0u;
    uint32_t a = dot(v.x, w, c.acc);
    uint32_t b = dot(v.y, w, 0u);
    a = dot(v.z, w, a);
    b = dot(v.w, w, b);
    c.acc = a + b;
  } else {  // some lane holds a frame's partial last chunk: byte masks
    // (an odd end leaves the last word's high byte 0, as the reference pads)
    const uint32_t f = live ? 0xffffffffu : 0u;
    const uint4 mm = part ? c.m : make_uint4(f, f, f, f);
    uint32_t a = dot(v.x & mm.x, 0x00010001u, c.acc);
    uint32_t b = dot(v.y & mm.y, 0x00010001u, 0u);
    a = dot(v.z & mm.z, 0x00010001u, a);
    b = dot(v.w & mm.w, 0x00010001u, b);
    c.acc = a + b;
  }
  if (++c.rnd == c.R) {  // the slot's jobs end: fold each group
    const uint32_t t = group_sum8(c.acc);
    if ((lane & 7u) == c.js) c.bs = t;
    c.acc = 0;
    consume_slot(c, J, c.js + 1, lane);
  }
}

#endif  // OO_RX_GSEQ

// Tiles.  The batch is cut into P.ntiles tiles, K per tile-processing wave
// (rx_kernel's waves), which take tiles w, w + W, ...
// (all waves sweep the buffer together: reading one ~200-MB window at a time
// is faster than 2560 separate contiguous ranges).  Tile sizes are multiples
// of 8 -- tlo or tlo + 8 packets, the last tile taking the < 8 left over --
// so the body stream's job slots fill (a slot holds 8 jobs).
struct Unit {
  uint32_t first, cnt;  // packets [first, first + cnt)
  uint32_t key;         // spreads the tile's zero lines
};
__device__ __forceinline__ Unit unit_of(const KParams& P, uint32_t t) {
  Unit u;
  u.key = t;
  if (t >= P.ntiles) {
    u.first = 0;
    u.cnt = 0;
    return u;
  }
  u.first = P.tlo * t + P.tstep * min(t, P.ta);
  u.cnt = t + 1u == P.ntiles ? P.n - u.first : P.tlo + (t < P.ta ? P.tstep : 0u);
  return u;
}

// A unit's zero lines: 1 KiB of the zero region per unit, so the lanes that
// read zeros are spread over the L2 channels.
__device__ __forceinline__ uint64_t zero_line(const KParams& P, const Unit& t, uint32_t lane) {
  return reinterpret_cast<uint64_t>(P.zero) +
         (uint64_t)(((t.key * 64u + lane) & (ZERO_LINES - 1u)) * 16u);
}

// ---------------------------------------------------------------------------

// A tile's descriptor as seen by its lane: frame start, its 16-B-aligned base
// and span, all 0 for lanes without a packet or out-of-buffer descriptors.
struct DescView {
  uint64_t abase;
  int shift, len, span, intf_i;
  bool valid;
  uint32_t idx;
};
__device__ __forceinline__ DescView desc_view(const KParams& P, const uint4& d, const Unit& t,
                                              uint32_t lane) {
  DescView v;
  v.idx = t.first + lane;
  v.valid = lane < t.cnt;
  // Both layouts: {u64 offset, 16-bit length, ...}.  An AF_XDP entry's u32
  // len is carried in ef_event's 16-bit rx.len (ef_vi.h:154,
  // efxdp_vi.c:349), and its frame starts at UMEM + addr: buffer addr / 2048
  // at offset addr & 2047 (efxdp_vi.c:337-348, netif_event.c:1723-1727).
  const uint64_t off = (uint64_t)d.x | ((uint64_t)d.y << 32);
  int len = (int)(d.z & 0xffffu);
  v.intf_i = P.xdp ? P.xdp_intf : (int)(int16_t)(d.z >> 16);
  // In bounds, without the u64 wrap of off + len (an offset near 2^64 must
  // not land before the buffer).
  const bool inb = v.valid && off <= P.frames_bytes && (uint64_t)len <= P.frames_bytes - off;
  if (!inb) len = 0;  // a descriptor outside the buffer is an empty frame
  const uint64_t base = reinterpret_cast<uint64_t>(P.frames) + (inb ? off : 0);
  v.shift = (int)(base & 15u);
  v.abase = base - (uint64_t)v.shift;
  v.len = len;
  v.span = inb ? v.shift + len : 0;
  return v;
}

// Where lane `lane` of unit t loads its descriptor from (lanes without a
// packet: some other in-bounds entry).
__device__ __forceinline__ uint64_t desc_base(const KParams& P) {
  return reinterpret_cast<uint64_t>(P.desc);
}
__device__ __forceinline__ uint64_t desc_at(const KParams& P, uint32_t i) {
  return desc_base(P) + (uint64_t)((P.ring_cons + i) & P.ring_mask) * 16;
}
__device__ __forceinline__ uint64_t desc_src(const KParams& P, const Unit& t, uint32_t lane) {
  return desc_at(P, lane < t.cnt ? t.first + lane : lane % P.n);
}

// Stages the tile's header windows for the parse.  Rows 0..HC-1 hold the
// windows packet-major: packet p's 128-B window is row-major at byte 128 p,
// its cell k at 16 * ((k - p) & 7) within it, so one LDS-DMA instruction
// reads eight packets' windows, eight lanes (one 128-B run) per packet --
// 8-16 cache lines per instruction, not 64 -- and the packet-per-lane reads
// of any one cell fall in distinct banks.  Chunks a frame does not have read
// zeros.  All lanes active.
template <int AUX = OO_RX_HDR_AUX>
__device__ __forceinline__ void stage_window(const DescView& dv, uint64_t zero, uint4 (*rows)[64],
                                             uint32_t lane, bool masked = false) {
  const uint32_t lo = (uint32_t)dv.abase, hi = (uint32_t)(dv.abase >> 32);
  // Every row's frame fields first (24 permutes, one wait), then the eight
  // DMAs: fetched row by row, each row waited for its own permutes.
  uint32_t l[HC], h[HC], sp[HC];
#pragma unroll
  for (int i = 0; i < HC; ++i) {
    const uint32_t p = (uint32_t)i * 8u + (lane >> 3);
    l[i] = lane_get(lo, p);
    h[i] = lane_get(hi, p);
    sp[i] = lane_get((uint32_t)dv.span, p);
  }
#pragma unroll
  for (int i = 0; i < HC; ++i) {
    const uint32_t p = (uint32_t)i * 8u + (lane >> 3);
    const uint32_t c = ((lane & 7u) + p) & 7u;
    const uint64_t ab = (uint64_t)h[i] << 32 | l[i];
    const int nwin = ((int)sp[i] + 15) >> 4;
    // masked (wave-uniform): cells 4..7 already hold zeros and no frame has
    // them -- those lanes issue nothing (lane 0 reads cell 0: every row is
    // still one instruction).
    if (!masked || c < 4u) glds<AUX>((int)c < nwin ? ab + (uint64_t)c * 16 : zero, &rows[i][0]);
  }
}

__device__ __forceinline__ Win window_of(uint4 (*rows)[64], uint32_t lane) {
  Win W;
  W.row = reinterpret_cast<const uint8_t*>(&rows[0][0]) + 128u * lane;
  W.rot = (8u - (lane & 7u)) & 7u;
  return W;
}

// ---------------------------------------------------------------------------
// TX checksum fill: oo_pkt_calc_checksums
// (src/lib/transport/ip/pkt_checksum.c:20-102) as calc_csum_if_needed
// (netif_tx.c:24-40) calls it, on the same streaming engine.  Only TCP and
// UDP frames: the IPv4 header checksum (ef_ip_checksum, checksum.c:185-212),
// then the L4 check field over the L4 header and the rest of the frame
// (ef_udp_checksum{,_ip6} checksum.c:225-250, not for an IPv4 fragment;
// ef_tcp_checksum{,_ip6} checksum.c:260-296).  The L4 sum here covers the
// whole L4 region including the old check field, and the pseudo-header term
// carries 0xffff - old check, which is what the reference's TCP code does and
// is the same value mod 0xffff as the UDP code's skipping of the field; both
// sums are non-zero (the pseudo-header holds the protocol), so the folds
// agree.  A frame whose headers do not fit, or with IHL < 5 or TCP doff < 5,
// keeps its L4 check field (and, when the IPv4 header itself does not fit or
// has IHL < 5, its IP check field) -- the reference asserts those away.

struct TxHdr {
  uint32_t ip_pos, l4_pos;  // frame offsets of the check fields
  uint32_t ip_ck;           // the IPv4 header checksum to store
  bool ip_do, l4_do, udp, longl4;
  bool whole;       // fixed format, 64-B-aligned frame of >= 64 B: its first 64 B
  uint4 head[4];    //   (as staged) are written back whole, check fields patched
  uint32_t s4;      // window part of the L4 region's word sum (window coordinates)
  uint32_t pseudo;  // pseudo-header words + 0xffff - old check (L4-relative)
};

// The fixed-format TX header (16-B-aligned start, untagged IPv4 IHL 5, TCP
// or UDP whose header fits): fields at fixed offsets from the staged cells,
// the same decisions as tx_general.  false: another frame.
__device__ __forceinline__ bool tx_fixed(const uint4 (&c)[HC], int shift, int len, int off0,
                                         TxHdr& h) {
  const uint32_t proto = c[1].y >> 24;
  const bool tcp = proto == 6u;
  const uint32_t doff4 = ((c[2].w >> 20) & 0xfu) * 4u;
  bool ok = shift == 0 && off0 >= 48 && len >= 48 && (c[0].w & 0x000fffffu) == 0x00050008u &&
            (tcp || proto == 17u);
  ok = ok && (tcp ? (len >= 54 && doff4 >= 20u && (uint32_t)len >= 34u + doff4) : len >= 42);
  if (!ok) return false;
  // A write of part of a 64-B memory granule is read-modify-written by the
  // memory; the frame's first granule, holding both check fields, is
  // therefore written back whole when it lies inside the frame.
  h.whole = len >= 64 && (off0 & 63) == 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) h.head[k] = c[k];
  const uint32_t frag = bswap16(c[1].y);
  const uint32_t addrs = (c[1].z >> 16) + (c[1].w & 0xffffu) + (c[1].w >> 16) + (c[2].x & 0xffffu);
  // IPv4 header words, bytes [14, 34) without the check field [24, 26).
  h.ip_do = true;
  h.ip_pos = 24;
  h.ip_ck = (~fold16(chunk_sum_all(c[1], (c[0].w >> 16) + (c[2].x & 0xffffu)) -
                     (c[1].z & 0xffffu))) & 0xffffu;
  h.udp = !tcp;
  h.l4_do = tcp || (frag & ~0x4000u) == 0u;
  if (tcp) {
    const uint32_t pl = (bswap16(c[1].x) - 20u) & 0xffffu;
    h.l4_pos = 50;
    h.pseudo = addrs + 0x0600u + bswap16(pl) + (0xffffu - (c[3].x >> 16));
  } else {
    h.l4_pos = 40;
    h.pseudo = addrs + 0x1100u + (c[2].y >> 16) + (0xffffu - (c[2].z & 0xffffu));
  }
  // L4 window part [34, E4h), as parse_fixed.
  const int E4 = len;
  h.longl4 = E4 > HB;
  const int E4h = h.longl4 ? off0 : E4;
  uint32_t s4 = 0;
  if (__ballot((E4h & 15) != 0) == 0) {
#pragma unroll
    for (int k = 2; k < HC; ++k) {
      const uint32_t t = chunk_sum_all(c[k], 0u);
      s4 += E4h >= 16 * k + 16 ? t : 0u;
    }
    s4 -= E4h >= 48 ? (c[2].x & 0xffffu) : 0u;
  } else {
#pragma unroll
    for (int k = 2; k < HC; ++k)
      if (16 * k < E4h) s4 += chunk_sum(c[k], 16 * k, 34, E4h);
  }
  h.s4 = s4;
  return true;
}

__device__ __forceinline__ TxHdr tx_general(const Win& W, int shift, int len, uint64_t abase) {
  auto B = [&](int j) -> uint32_t {
    int w = shift + j;
    w = w < HB ? w : HB - 1;
    const uint32_t v = W.cell(w >> 4)[w & 15];
    return j < len ? v : 0u;
  };
  auto BE16 = [&](int j) -> uint32_t { return (B(j) << 8) | B(j + 1); };
  auto N16 = [&](int j) -> uint32_t { return B(j) | (B(j + 1) << 8); };
  TxHdr h;
  h.ip_do = h.l4_do = h.udp = h.longl4 = h.whole = false;
  h.ip_pos = h.l4_pos = h.ip_ck = h.s4 = h.pseudo = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) h.head[k] = make_uint4(0, 0, 0, 0);
  if (len < 14) return h;
  const int l3 = BE16(12) == 0x8100u ? 18 : 14;  // ci_parse_rx_vlan
  const uint32_t et = BE16(l3 - 2);
  const bool af6 = et == 0x86ddu;
  if (!af6 && et != 0x0800u) return h;
  int ihl4 = 40;
  uint32_t proto;
  if (!af6) {
    if (len < l3 + 20) return h;
    ihl4 = (int)(B(l3) & 0xfu) * 4;
    if (ihl4 < 20 || len < l3 + ihl4) return h;
    proto = B(l3 + 9);
  } else {
    if (len < l3 + 40) return h;
    proto = B(l3 + 6);
  }
  if (proto != 6u && proto != 17u) return h;
  const int l4 = l3 + ihl4;
  if (!af6) {  // ef_ip_checksum: the header words without the check field
    uint32_t s = 0;
    for (int k = 0; k < ihl4; k += 2) s += k == 10 ? 0u : N16(l3 + k);
    h.ip_do = true;
    h.ip_pos = (uint32_t)(l3 + 10);
    h.ip_ck = (~fold16(s)) & 0xffffu;
  }
  uint32_t pseudo = 0;
  int ck;
  if (proto == 17u) {
    if (!af6 && (BE16(l3 + 6) & ~0x4000u) != 0) return h;  // ci_ipx_is_frag
    if (len < l4 + 8) return h;
    ck = l4 + 6;
    pseudo = 0x1100u + N16(l4 + 4);
  } else {
    if (len < l4 + 20) return h;
    const int hl4 = (int)(B(l4 + 12) >> 4) * 4;
    if (hl4 < 20 || len < l4 + hl4) return h;
    ck = l4 + 16;
    if (af6) {
      pseudo = 0x0600u + N16(l3 + 4);
    } else {
      const uint32_t pl = (BE16(l3 + 2) - (uint32_t)ihl4) & 0xffffu;
      pseudo = 0x0600u + (((pl & 0xffu) << 8) | (pl >> 8));
    }
  }
  if (af6) {
#pragma unroll
    for (int i = 0; i < 16; ++i) pseudo += N16(l3 + 8 + 2 * i);
  } else {
    pseudo += N16(l3 + 12) + N16(l3 + 14) + N16(l3 + 16) + N16(l3 + 18);
  }
  h.pseudo = pseudo + (0xffffu - N16(ck));
  h.l4_do = true;
  h.udp = proto == 17u;
  h.l4_pos = (uint32_t)ck;
  // The L4 region is [l4, len): its window part, as on RX (the body stream
  // covers [off0, span) when the region runs past the window).
  const int off0 = (int)body_off0(abase);
  const int S4 = shift + l4, E4 = shift + len;
  h.longl4 = E4 > HB;
  const int cut = h.longl4 ? off0 : E4;
  const int lo4 = min(S4, cut), hi4 = max(S4, cut);
  uint32_t s4 = 0;
#pragma unroll
  for (int k = 0; k < HC; ++k) {
    if (k * 16 < hi4) s4 += chunk_sum(*reinterpret_cast<const uint4*>(W.cell(k)), k * 16, lo4, hi4);
  }
  h.s4 = cut < S4 ? 0u - s4 : s4;
  return h;
}

__device__ __forceinline__ TxHdr tx_header(const Win& W, int shift, int len, uint64_t abase) {
  TxHdr h;
  bool fixed;
  {
    uint4 c[HC];
    read_cells(W, c);
    fixed = tx_fixed(c, shift, len, (int)body_off0(abase), h);
  }
  if (__ballot(!fixed) != 0) {
    if (!fixed) h = tx_general(W, shift, len, abase);
  }
  return h;
}

// The L4 check value from the window part, the body sum and the
// pseudo-header term (ip_proto_csum64_finish; UDP 0 -> 0xffff).
__device__ __forceinline__ uint32_t tx_l4_check(const TxHdr& h, int shift, uint32_t body) {
  uint32_t f = fold16(h.s4 + (h.longl4 ? body : 0u));
  if (shift & 1) f = swap16(f);  // RFC 1071 byte-order swap
  const uint32_t v = (~fold16(f + h.pseudo)) & 0xffffu;
  return (h.udp && v == 0u) ? 0xffffu : v;
}

__device__ __forceinline__ void lds_write16(void* p, const uint4& v) {
  const u32x4 w = {v.x, v.y, v.z, v.w};
  asm volatile("ds_write_b128 %0, %1" ::"v"((uint32_t)(uintptr_t)(lptr)(p)), "v"(w) : "memory");
}

// The wave's NST_TX = 6 stores (tests/test_kernel_isa.py checks the code
// object holds exactly these).  Frames in the whole-granule form (TxHdr):
// their first 64 B with the check fields patched in (fixed format: IPv4
// check at 24, UDP at 40, TCP at 50), staged through the idle ring so that
// store u writes the granules of frames 16u .. 16u + 15, four lanes per
// granule -- whole 64-B writes.  Every other frame: the two check fields as
// 16-bit stores (little-endian, as the reference's u16 stores; the address
// may be odd).  Lanes with nothing to write store to the sink, so the count
// is static.  All stores are global-address-space (a flat store would count
// in lgkmcnt too).  All lanes active; the ring holds no DMA (the body stream
// has drained).
typedef __attribute__((address_space(1))) u32x4 g_u32x4;
typedef __attribute__((address_space(1))) uint16_t g_uint16;
__device__ __forceinline__ void gstore16(uint64_t a, const uint4& v) {
  const u32x4 w = {v.x, v.y, v.z, v.w};
  *reinterpret_cast<g_u32x4*>(a) = w;
}
__device__ __forceinline__ void gstore2(uint64_t a, uint32_t v) {
  *reinterpret_cast<g_uint16*>(a) = (uint16_t)v;
}
constexpr int NST_TX = 6;
#if !defined(OO_RX_SHORT)
static_assert(R >= 4, "store_checks stages 64 lanes x 64 B in the ring");
#endif
__device__ __forceinline__ void store_checks(const KParams& P, const DescView& dv,
                                             const TxHdr& h, uint32_t l4v, uint32_t lane,
                                             uint4 (*ring)[64]) {
  uint8_t* const frame = reinterpret_cast<uint8_t*>(dv.abase + (uint64_t)dv.shift);
  uint8_t* const sink = P.sink + 4u * lane;
  const bool whole = dv.valid && h.whole;
  const bool ip = dv.valid && !h.whole && h.ip_do, l4 = dv.valid && !h.whole && h.l4_do;
  {
    uint4 hd[4] = {h.head[0], h.head[1], h.head[2], h.head[3]};
    hd[1].z = (hd[1].z & 0xffff0000u) | h.ip_ck;
    if (h.l4_do) {
      if (h.udp) hd[2].z = (hd[2].z & 0xffff0000u) | l4v;
      else hd[3].x = (hd[3].x & 0xffffu) | (l4v << 16);
    }
    // Lane p's 64 B at ring byte 64 p.
#pragma unroll
    for (int k = 0; k < 4; ++k) lds_write16(&ring[lane >> 4][((lane * 4u) & 63u) + k], hd[k]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint64_t fa = reinterpret_cast<uint64_t>(frame);
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) {
      const uint32_t f = 16u * u + (lane >> 2);
      const uint4 v = lds_read16(&ring[u][lane]);
      const bool wf = lane_get(whole ? 1u : 0u, f) != 0;
      const uint64_t a = (uint64_t)lane_get((uint32_t)fa, f) |
                         ((uint64_t)lane_get((uint32_t)(fa >> 32), f) << 32);
      gstore16(wf ? a + 16u * (lane & 3u) : reinterpret_cast<uint64_t>(P.sink) + 16u * lane, v);
    }
  }
  uint8_t* const pi = ip ? frame + h.ip_pos : sink;
  uint8_t* const pl = l4 ? frame + h.l4_pos : sink + 2;
  gstore2(reinterpret_cast<uint64_t>(pi), h.ip_ck);
  gstore2(reinterpret_cast<uint64_t>(pl), l4v);
}

// ---------------------------------------------------------------------------
// rx_kernel: every wave parses and streams its own tiles, software-pipelined:
// while a tile's body streams, the next tile's header windows (and the
// descriptors of the tile after it) land in LDS, so each tile starts with its
// headers in place.  A wave's vector-memory operations (loads, LDS-DMA,
// stores) retire in issue order, and every wait counts the operations issued
// after the ones it needs: NHS staging operations per tile (HC header rows,
// one descriptor line and the tile claim) and NST record stores, all issued
// by the wave whatever its lanes hold, so the counts are static.
//
// Tiles are handed out dynamically: a wave's first three tiles are gwave +
// k W (k < 3), every later one comes from a counter (claim_tile), claimed
// three tiles ahead -- the descriptors are prefetched two tiles ahead -- so
// a wave that runs fast takes more tiles and the waves finish together (the
// host cuts the batch's end into small tiles, launch()).  Atomics on one
// address serialise (~12 ns each), so the waves are split into P.ngroups
// groups (gwave mod ngroups, spread over all CUs), each with its own counter
// over its own tiles (those = its group mod ngroups).
// A stream's launches alternate between two counter sets, each launch
// zeroing the set of the next one as it starts, so a wave ends with its last
// record stores: nothing waits for the group's other claims.

constexpr int NHS = HC + 2;
constexpr int NST = 2;
// Extra body rounds a long tile puts in flight in the header rows once the
// parse has read them (the header work then overlaps E more KiB of stream).
#ifndef OO_RX_EXTRA
#define OO_RX_EXTRA 8
#endif
constexpr int E = OO_RX_EXTRA;
static_assert(E % 2 == 0 && E <= HC, "extra rounds live in the header rows");

struct WaveLds {
  uint4 hdr[HC][64];            // header windows (stage_window)
  uint4 ring[R][64];            // body ring: slot = one round of the eight groups
  uint4 desc[2][64];            // descriptors of this tile and of the next
  uint32_t cnt[OO_RX_R_COUNT];  // per-reason counts
  uint32_t dbase, gofs;          // claims: first dynamic tile of the group, counter offset
  uint32_t T0, pad;              // the tile's body rounds (kept out of the registers)
};
static_assert(sizeof(WaveLds) % 16 == 0, "WaveLds is carved from a uint4 array");
constexpr int WAVE_U4 = (int)(sizeof(WaveLds) / 16);

__device__ __forceinline__ void lds_write4(void* p, uint32_t v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"((uint32_t)(uintptr_t)(lptr)(p)), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_add4(void* p, uint32_t v) {
  asm volatile("ds_add_u32 %0, %1" ::"v"((uint32_t)(uintptr_t)(lptr)(p)), "v"(v) : "memory");
}
__device__ __forceinline__ uint32_t lds_read4(const void* p) {
  uint32_t v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)"
               : "=v"(v)
               : "v"((uint32_t)(uintptr_t)(lptr)(p))
               : "memory");
  return v;
}

// vm_wait with a count that is a constant only after unrolling.
__device__ __forceinline__ void vm_wait_n(int n) {
  switch (n) {
#define OO_W(k) \
  case k:       \
    vm_wait<k>(); \
    break;
    OO_W(0) OO_W(1) OO_W(2) OO_W(3) OO_W(4) OO_W(5) OO_W(6) OO_W(7) OO_W(8) OO_W(9) OO_W(10)
    OO_W(11) OO_W(12) OO_W(13) OO_W(14) OO_W(15) OO_W(16) OO_W(17) OO_W(18) OO_W(19) OO_W(20)
    OO_W(21) OO_W(22) OO_W(23) OO_W(24) OO_W(25) OO_W(26) OO_W(27) OO_W(28) OO_W(29) OO_W(30)
#undef OO_W
    default:
      vm_wait<0>();
  }
}

// The tile's records (packet p's in lane p): the wave writes them as two
// contiguous 1-KiB runs, store u taking records 32u .. 32u + 31 with lane L
// writing half L & 1 of record 32u + L / 2 -- whole lines per instruction,
// not 16 B at a 32-B stride.  Lanes past the tile's count write the tile's
// last record again (the same bytes to the same address), so the wave always
// issues exactly NST stores and needs no per-lane sink address (tiles are
// never empty: the host's partition, oo_gpu_rx.cpp launch()).  All lanes
// active.
// DIRECT: each lane stores its own record (two 16-B stores at a 32-B
// stride; win_kernel: config 3 -2.5 %) instead of the lane-permuted 1-KiB
// runs (rx_kernel, where the direct form measured +1.2 % on config 2:
// profiles/r06/ab_rec_direct_c2-5.log).
template <bool DIRECT = false>
__device__ __forceinline__ void store_records(const KParams& P, const Unit& t,
                                              const oo_gpu_rx_result& r, uint32_t lane) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&r);
  const uint32_t hi = lane & 1u;
  const uint32_t last = t.cnt - 1u;
  // (a global pointer whatever P.out came from -- HBM or host-mapped
  // records: a generic pointer would make these flat stores, counted in
  // lgkmcnt as well)
  __attribute__((address_space(1))) u32x4* const out =
      (__attribute__((address_space(1))) u32x4*)reinterpret_cast<uintptr_t>(P.out);
  if constexpr (DIRECT) {
    if (lane < t.cnt) {
      out[(size_t)(t.first + lane) * 2u] = u32x4{w[0], w[1], w[2], w[3]};
      out[(size_t)(t.first + lane) * 2u + 1u] = u32x4{w[4], w[5], w[6], w[7]};
    }
    return;
  }
#pragma unroll
  for (uint32_t u = 0; u < 2; ++u) {
    const uint32_t q = min(32u * u + (lane >> 1), last);
    uint4 v;
    uint32_t* vw = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const uint32_t a = lane_get(w[d], q), b = lane_get(w[4 + d], q);
      vw[d] = hi ? b : a;
    }
    out[(size_t)(t.first + q) * 2u + hi] = u32x4{v.x, v.y, v.z, v.w};
  }
}

// One tile claim: lane 0 adds 1 to the launch's counter and gets the old
// value back in `got` (one returning global atomic: one vector-memory
// operation of the wave, counted like the others).  The compiler tracks the
// result and waits for it where it is read, a tile later.
__device__ __forceinline__ void claim_tile(uint32_t* ctr, uint32_t step, uint32_t lane,
                                           uint32_t& got) {
  if (lane == 0) got = __hip_atomic_fetch_add(ctr, step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Zeroes the claim set the stream's next launch uses (its CLAIM_LINES lines:
// both kernels' group counters and the body flag) with three `sc1` stores;
// the launch before it, the last to use that set, has finished (stream
// order).
__device__ __forceinline__ void zero_claim_set(uint32_t* set, uint32_t lane) {
  static_assert(CLAIM_GROUPS == 64, "one lane per group counter");
  __hip_atomic_store(set + 32u * lane, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(set + 32u * (CLAIM_GROUPS + lane), 0u, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
  if (lane == 0)
    __hip_atomic_store(set + 32u * FLAG_LINE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The claim group of wave gwave: runs of B = 2^gshift consecutive waves
// (gshift 4: eight blocks, one on each XCD) dealt round-robin to the groups.
__device__ __forceinline__ uint32_t group_of(const KParams& P, uint32_t gwave) {
  return (gwave >> P.gshift) & (P.ngroups - 1u);
}

// The per-wave tile loop of rx_kernel (TX = false) and tx_kernel (TX =
// true): the same staging and body stream, different header work and stores.
template <bool TX>
__device__ __forceinline__ void tile_loop(const KParams& P) {
  constexpr int NSTK = TX ? NST_TX : NST;  // stores per tile
  // All LDS in one __shared__ array (a second object can make hipcc wait
  // vmcnt(0) before LDS reads while LDS-DMA is in flight).
  __shared__ __attribute__((aligned(16))) uint4 smem[WAVES * WAVE_U4];

  const int wave = (int)(threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63u;
  WaveLds& L = reinterpret_cast<WaveLds*>(smem)[wave];

  const uint32_t gwave = sreg(blockIdx.x * WAVES + wave);  // wave-uniform
  const uint32_t W = gridDim.x * WAVES;
  // The stream's launches alternate between two claim counter sets: this one
  // zeroes the set the next one will use (the launch before it, which left
  // that set's counters where its claims ended, has finished: stream order).
  // No wave has to wait for the others' claims at the end.
  if (gwave == 0) zero_claim_set(P.claim_next, lane);
  // Tiles i, i + 1, i + 2 of this wave, and the claim of tile i + 3.
  uint32_t tcur = gwave, tnext = gwave + W, tnext2 = gwave + 2u * W, got = 0;
  uint32_t claimed = 0;  // the last claim, once read (have)
  bool have = false;
  // Group g's claims are g + 3 W, g + 3 W + ngroups, ... (its counter holds
  // the multiple of ngroups handed out); kept in LDS, out of the registers.
  if (lane == 0) {
    const uint32_t g = group_of(P, gwave);
    lds_write4(&L.dbase, 3u * W + g);
    lds_write4(&L.gofs, 32u * g);
  }
  if (gwave < P.ntiles) {
  if (lane < OO_RX_R_COUNT) lds_write4(&L.cnt[lane], 0u);

  // Prologue: this tile's descriptors, then the next tile's and this tile's
  // header windows.
  const Unit t0 = unit_of(P, tcur);
  glds<0>(desc_src(P, t0, lane), &L.desc[0][0]);
  vm_wait<0>();
  glds<0>(desc_src(P, unit_of(P, tnext), lane), &L.desc[1][0]);
  {
    const DescView d0 = desc_view(P, lds_read16(&L.desc[0][lane]), t0, lane);
    stage_window(d0, zero_line(P, t0, lane), L.hdr, lane);
  }

  uint32_t b = 0, it_ = 0;
  for (; tcur < P.ntiles; b ^= 1u, ++it_) {
    STAMP(0, __builtin_amdgcn_s_memrealtime());
    const Unit tile = unit_of(P, tcur);
    STAMP(6, tile.first);
    const DescView dv = desc_view(P, lds_read16(&L.desc[b][lane]), tile, lane);
    const uint64_t zero = zero_line(P, tile, lane);

    // ---- body jobs; the first R rounds land during the parse.  A tile with
    // more than R + E rounds ("ext") also streams E rounds into the header
    // rows during the demux: rounds 0..R-1 ring, R..R+E-1 header rows,
    // R+E.. ring again; its next header windows are staged once the header
    // rows are consumed.  T: the ring-loop rounds (a multiple of R; the
    // padding rounds read zeros).
    uint32_t myslot;
    const Jobs J = jobs_setup(dv.abase, dv.span, lane, myslot);
#ifdef OO_RX_BOUND_NOBODY  // (a timing bound, wrong records: no body stream)
    uint32_t T0 = 0;
#else
    uint32_t T0 = J.T;
#endif
    bool ext = E > 0 && T0 > (uint32_t)(R + E);
    uint32_t T = ext ? (T0 - R - E + R - 1) / R * R : (T0 + R - 1) / R * R;
    if (lane == 0) lds_write4(&L.T0, T0);
    IssueCursor ci;
    if (T0 != 0) issue_slot(ci, J, 0, lane, zero);  // (body-less tiles issue no rounds)
    // This tile's header windows: older than the previous tile's NST stores
    // (none before the first tile) and the R rounds issued here.
    if (T != 0) {
#pragma unroll
      for (int u = 0; u < R; ++u) issue_round(ci, J, zero, &L.ring[u][0], lane);
      if (it_ == 0) vm_wait<R>();
      else vm_wait<R + NSTK>();
    } else {
      if (it_ == 0) vm_wait<0>();
      else vm_wait<NSTK>();
    }

    STAMP(1, __builtin_amdgcn_s_memrealtime());
    STAMP(7, T0);

    // Rounds R..R+E-1 into the header rows, once their windows are read --
    // and after the demux: issued before it they are older than its loads,
    // and every demux wait would wait for them too (configs 2/4/5 -1.7 /
    // -0.5 / -0.7 %, profiles/r04/ab_extra_after_demux.log).
    auto issue_extra = [&]() {
      if (ext) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int u = 0; u < E; ++u) issue_round(ci, J, zero, &L.hdr[u][0], lane);
      }
    };

    // ---- header work (one packet per lane).
    Parsed ps;
    TxHdr th;
    if constexpr (TX) {
      th = tx_header(window_of(L.hdr, lane), dv.shift, dv.len, dv.abase);
      issue_extra();
    } else {
#ifdef OO_RX_STAMPS
      if (lane == 0)
        dstamp_slot(P.stamps != nullptr && it_ < 128 ? &P.stamps[((size_t)gwave * 128 + it_) * 16] : nullptr,
                    true);
#endif
      const Hdr h = parse_headers<false>(window_of(L.hdr, lane), dv.shift, dv.len, dv.abase);
      STAMP(2, __builtin_amdgcn_s_memrealtime());
      ps = demux_packet(P, h, dv.intf_i, dv.abase, dv.span, dv.shift);
      issue_extra();
    }
    STAMP(3, __builtin_amdgcn_s_memrealtime());

    // ---- stage the next tile: descriptors of the tile after it into this
    // tile's buffer, its header windows (an ext tile: after its header-row
    // rounds), and the claim of the tile after that.
    T0 = sreg(lds_read4(&L.T0));
    ext = E > 0 && T0 > (uint32_t)(R + E);
    T = ext ? (T0 - R - E + R - 1) / R * R : (T0 + R - 1) / R * R;
    // Tile i + 2: the claim issued at the previous tile, read at its end
    // (have) or, after a tile without a body, here (the compiler waits for
    // it: vmcnt(0), which a body-less tile has little in flight to pay for).
    if (it_ != 0) {
      uint32_t c;
      if (have) {
        c = claimed;
      } else {
        asm volatile("" ::: "memory");  // keeps the read (and its wait) on this path
        c = (uint32_t)__builtin_amdgcn_readfirstlane((int)got);
      }
      tnext2 = P.dyn ? sreg(lds_read4(&L.dbase)) + c : tnext2 + W;
      have = false;
    }
    glds<0>(desc_src(P, unit_of(P, tnext2), lane), &L.desc[b][0]);
    auto stage_next = [&]() {
      const Unit nt = unit_of(P, tnext);
      const DescView dn = desc_view(P, lds_read16(&L.desc[b ^ 1u][lane]), nt, lane);
      stage_window(dn, zero_line(P, nt, lane), L.hdr, lane);
    };
    if (!ext) stage_next();

    claim_tile(P.claim + sreg(lds_read4(&L.gofs)), P.ngroups, lane, got);  // tile i + 3

    // The consume side's cursor is set up only now: its registers are free
    // during the header work, where the demux loads need them.
    ConsumeCursor cc;
    if (T0 != 0) {
      consume_start(cc, J, lane);
    } else {  // nothing to consume: every body sum is 0
      cc.acc = 0;
      cc.bs = 0;
    }

    // ---- body stream, two pieces per step.  Each wait counts the
    // operations issued after the awaited pair (the demux loads excepted:
    // the demux waited for its last one, and with it for everything older).
    if (ext) {
      // Ring rounds 0..R-1, refilled with R+E..R+E+R-1: newer than the
      // pair, the rest of the ring, the E header-row rounds, the descriptor
      // line and the claim, and the refills so far -- R + E in all.
#pragma unroll
      for (int u = 0; u < R; u += 2) {
        vm_wait<R + E>();
        uint4 v0, v1;
        lds_read16x2(&L.ring[u][lane], &L.ring[u + 1][lane], v0, v1);
        consume_round(cc, J, v0, lane);
        consume_round(cc, J, v1, lane);
        issue_round(ci, J, zero, &L.ring[u][0], lane);
        issue_round(ci, J, zero, &L.ring[u + 1][0], lane);
      }
      // Header-row rounds R..R+E-1: newer, the rest of them, the descriptor
      // line and the claim, and the R refills.
#pragma unroll
      for (int u = 0; u < E; u += 2) {
        vm_wait_n(R + E - u);
        uint4 v0, v1;
        lds_read16x2(&L.hdr[u][lane], &L.hdr[u + 1][lane], v0, v1);
        consume_round(cc, J, v0, lane);
        consume_round(cc, J, v1, lane);
      }
      stage_next();
    }
    // The ring loop (T is a multiple of R).  Newer than the awaited pair: the
    // rest of the ring, plus in the first turn the staging operations issued
    // since the ring was filled (NHS, or HC after an ext prefix); none past T.
    const int nhs = ext ? HC : NHS;
    for (uint32_t k0 = 0; k0 < T; k0 += R) {
      const bool first = k0 == 0, last = k0 + R == T;
#pragma unroll
      for (int u = 0; u < R; u += 2) {
        if (first && last) vm_wait_n(R - 2 - u + nhs);
        else if (first) vm_wait_n(R - 2 + nhs);
        else if (last) vm_wait_n(R - 2 - u);
        else vm_wait<R - 2>();
        uint4 v0, v1;
        lds_read16x2(&L.ring[u][lane], &L.ring[u + 1][lane], v0, v1);
        consume_round(cc, J, v0, lane);
        consume_round(cc, J, v1, lane);
        if (!last) {
          issue_round(ci, J, zero, &L.ring[u][0], lane);
          issue_round(ci, J, zero, &L.ring[u + 1][0], lane);
        }
      }
    }
    // The claim issued at this tile's staging has landed with the last body
    // round (the ring loop ends on vmcnt(0)): reading it here costs nothing.
    if (T != 0) {
      claimed = (uint32_t)__builtin_amdgcn_readfirstlane((int)got);
      have = true;
    }
    STAMP(4, __builtin_amdgcn_s_memrealtime());

    const uint32_t body = lane_get(cc.bs, myslot);
    if constexpr (TX) {
      store_checks(P, dv, th, tx_l4_check(th, dv.shift, body), lane, L.ring);
    } else {
      finish(ps, body);
      if (P.counters != nullptr && dv.valid)
        lds_add4(&L.cnt[ps.r.reason & (OO_RX_R_COUNT - 1)], 1u);
      store_records(P, tile, ps.r, lane);
    }
    STAMP(5, __builtin_amdgcn_s_memrealtime());
    tcur = tnext;
    tnext = tnext2;
  }

  // Per-reason counts: one global atomic per reason seen by the wave.  (The
  // lane index is recomputed: kept live across the loop it would spill.)
  const uint32_t ln = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  if (!TX && P.counters != nullptr) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (ln < OO_RX_R_COUNT) {
      const uint32_t c = lds_read4(&L.cnt[ln]);
      if (c != 0) atomicAdd(&P.counters[ln], c);
    }
  }
  }  // gwave < P.ntiles
}

#ifdef OO_RX_POLL
// ---------------------------------------------------------------------------
// The poll instance (oo_rx_kernel_poll.hip): a poll's batch
// of at most a few thousand packets, its frames often read in place over
// PCIe, is bound by its chain of round trips, not by bytes.  The same tile
// loop, with a ring deep enough (OO_RX_RING 12) that a tile of eight
// 1514-B frames issues its whole body with its header windows -- one round
// trip for the frames, where the 4-slot ring waits three -- and its own
// completion: each wave, once its record stores have completed, counts
// itself in the launch's claim-set FLAG_LINE word (zeroed by the stream's
// previous launch), and the last one writes the caller's done word in host
// memory -- no second operation on the stream after the kernel.
__device__ __forceinline__ void poll_done(const PollArgs& A) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  if (lane == 0) {
    const uint32_t prev =
        __hip_atomic_fetch_add(A.done_ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
    if (prev + 1u == gridDim.x * (uint32_t)WAVES)
      __hip_atomic_store(A.done, A.done_val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// (Few waves per launch: no occupancy target; the deep ring's unrolled
// rounds take more registers than three waves per SIMD allow.)
__global__ __launch_bounds__(WAVES * 64) void rx_kernel(PollArgs A) {
  tile_loop<false>(A.P);
  if (A.done != nullptr) poll_done(A);
}

#else
__global__ __launch_bounds__(WAVES * 64) __attribute__((amdgpu_waves_per_eu(3))) void rx_kernel(KParams P) {
  tile_loop<false>(P);
}
#endif
#ifndef OO_RX_POLL
#ifndef OO_RX_SHORT
__global__ __launch_bounds__(WAVES * 64) __attribute__((amdgpu_waves_per_eu(3))) void tx_kernel(KParams P) {
  tile_loop<true>(P);
}

// ===========================================================================
// The split transform (DESIGN.md §2 "Two launches"): a batch is two
// launches on its stream.
//  win_kernel   the header work of every packet -- descriptor, window
//               staging, parse, demux -- and every record, final unless the
//               L4 verdict waits for the frame's body (then written as if
//               the body sum passes); for the tiles holding frames with a
//               body, one 8-B pending word per packet (KParams::pend).
//  body_kernel  the bodies of the frames whose verdict waits, streamed by
//               the body engine above with nothing else in the wave's memory
//               queue; a frame whose sum fails gets the drop record that
//               finish() would have written.
// The records (2 % of config 2's bytes) are then written in win_kernel's
// short launch instead of between the body stream's reads: HBM pays for
// interleaved writes about a tenth of the stream's time.

// The body residue mod M = 0xffff for which the L4 verdict passes.  finish()
// passes iff fold16(f + pseudo) == 0xffff with f = fold16(s4 + body),
// byte-swapped for an odd frame address; a byte swap multiplies by 2^8 mod M
// and fold16 keeps the residue, so (pseudo >= 1: the sum is never 0) that is
// sigma (s4 + body) + pseudo == 0 (mod M), sigma = 256 or 1, i.e. body ==
// -s4 - sigma pseudo (mod M) (sigma^2 == 1 mod M).  s4 is the window part
// as the parse leaves it, possibly negative ("Why the split sum is exact";
// |s4| < 2^31: at most a 64-KiB frame's words).
#endif  // !OO_RX_SHORT
__device__ __forceinline__ uint32_t res16(uint32_t x) {  // x mod 0xffff
  const uint32_t f = fold16(x);
  return f == 0xffffu ? 0u : f;
}
#ifndef OO_RX_SHORT
__device__ __forceinline__ uint32_t body_target(uint32_t s4, uint32_t pseudo, bool odd) {
  const int32_t sv = (int32_t)s4;
  const uint32_t r4 = sv >= 0 ? res16((uint32_t)sv) : (0xffffu - res16((uint32_t)(-(int64_t)sv))) % 0xffffu;
  uint32_t rp = res16(pseudo);
  if (odd) rp = res16(rp << 8);
  return (2u * 0xffffu - r4 - rp) % 0xffffu;
}

constexpr int WAVES_W = 4;  // win_kernel: waves per block (sharing one bitmap copy)
#ifndef OO_RX_WIN_WPE
#define OO_RX_WIN_WPE 3  // win_kernel: waves per SIMD (LDS allows three 4-wave blocks per CU)
#endif

// 10 KiB a wave (the per-reason counts and the claim group stay in
// registers, reason_hist), plus the block's bitmap copy: 50 KiB a block, three
// blocks (12 waves) per CU.
struct WinLds {
  uint4 hdr[HC][64];             // header windows (stage_window)
  uint4 desc[2][64];             // descriptors of tile t (buffer t & 1) and t + 1
};
static_assert(sizeof(WinLds) == 10240, "10 KiB a wave");
constexpr int WIN_U4 = (int)(sizeof(WinLds) / 16);
constexpr int OCC_U4 = (int)((OCC_LDS_BYTES + 15) / 16);

// Lane k < 32: how many lanes of `valid` have reason k (five ballots of the
// reason's bits; the lane's own bits select each ballot or its complement).
__device__ __forceinline__ uint32_t reason_hist(uint32_t reason, bool valid, uint32_t lane) {
  static_assert(OO_RX_R_COUNT == 32, "five reason bits");
  uint64_t m = __ballot(valid);
  // (the common tile: every packet delivered -- one count, in lane 0)
  if (__ballot(valid && reason != OO_RX_R_DELIVER) == 0)
    return lane == 0 ? (uint32_t)__popcll(m) : 0u;
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const uint64_t bj = __ballot((reason >> j) & 1u);
    m &= ((lane >> j) & 1u) ? bj : ~bj;
  }
  return (uint32_t)__popcll(m);
}

// win_kernel's tile loop.  The same tiles, descriptor and window staging,
// parse, demux and claims as tile_loop, without a body: while tile t's
// lookups run, tile t+1's windows land (staged before the demux: its first
// level's wait then also covers them, one latency for both), and the
// descriptors of tile t+2 (into the buffer tile t's came in: read at the
// tile's start).  Counted waits, as tile_loop ("rx_kernel" above): per tile
// HC window rows, one descriptor line and the claim, then the demux loads
// (each level ends in vmcnt(0)), then NST record stores, and -- only for
// tiles holding a frame with a body -- the pending words (uncounted: an
// operation the count leaves out only makes a wait stricter).
__device__ __forceinline__ void window_loop(const KParams& P) {
  __shared__ __attribute__((aligned(16))) uint4 smem[WAVES_W * WIN_U4 + OCC_U4];
  const int wave = (int)(threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63u;
  WinLds& L = reinterpret_cast<WinLds*>(smem)[wave];
  // The block's copy of the occupancy bitmaps and hwport bytes (before any
  // LDS-DMA; the host sends only tables that fit, OCC_LDS_MAX4 / _MAX6).
  uint32_t* const occ = reinterpret_cast<uint32_t*>(smem + WAVES_W * WIN_U4);
  {
    const uint32_t n4 = (P.ip4_mask + 32u) >> 5, n6 = (P.ip6_mask + 32u) >> 5;
    for (uint32_t i = threadIdx.x; i < n4; i += WAVES_W * 64) occ[i] = P.occ4[i];
    for (uint32_t i = threadIdx.x; i < n6; i += WAVES_W * 64) occ[OCC_LDS_B6 / 4 + i] = P.occ6[i];
    if (threadIdx.x < 8)
      occ[OCC_LDS_HW / 4 + threadIdx.x] = reinterpret_cast<const uint32_t*>(P.hwport)[threadIdx.x];
    __syncthreads();
  }
  const uint32_t lds_occ = (uint32_t)(uintptr_t)(lptr)occ;
  const uint32_t gwave = sreg(blockIdx.x * WAVES_W + wave);
  const uint32_t W = gridDim.x * WAVES_W;
  if (gwave == 0) zero_claim_set(P.claim_next, lane);
  uint32_t tcur = gwave, tnext = gwave + W, tnext2 = gwave + 2u * W, got = 0;
  const uint32_t g = sreg(group_of(P, gwave));
  if (gwave >= P.ntiles) return;
  uint32_t cnt = 0;    // lane k < 32: this wave's count of reason k
  bool waits = false;  // a frame of this wave's tiles waits for its body

  // Window positions of cells 4..7 all zero (the last staged tile had no
  // frame past 64 bytes): a tile of such frames then stages cells 0..3 only.
#ifndef OO_RX_WIN_MASKED
#define OO_RX_WIN_MASKED 1
#endif
// The window rows of a tile whose frames all fit their windows are read
// nontemporal (read once, no body pass after them): config 3 -1.7 %.  A
// tile with longer frames keeps the default policy: body_kernel reads the
// rest of those lines (nontemporal there: config 5 +5 %; rx_kernel likewise
// keeps it, +11 % on config 2 with nontemporal header rows).
#ifndef OO_RX_WIN_HDR_AUX
#define OO_RX_WIN_HDR_AUX 2
#endif
#ifndef OO_RX_WIN_REC_DIRECT
#define OO_RX_WIN_REC_DIRECT 1  // each lane stores its own record (store_records)
#endif
  bool clean = false;
  // Prologue: tile t0's descriptors, then t1's and t0's windows.
  {
    const Unit t0 = unit_of(P, tcur);
    glds<0>(desc_src(P, t0, lane), &L.desc[0][0]);
    vm_wait<0>();
    glds<0>(desc_src(P, unit_of(P, tnext), lane), &L.desc[1][0]);
    const DescView d0 = desc_view(P, lds_read16(&L.desc[0][lane]), t0, lane);
    stage_window<OO_RX_HDR_AUX>(d0, zero_line(P, t0, lane), L.hdr, lane);
    clean = __ballot(d0.span > 64) == 0;
  }

  uint32_t b = 0;
  for (uint32_t it_ = 0; tcur < P.ntiles; b ^= 1u, ++it_) {
    const Unit tile = unit_of(P, tcur);
    // This tile's windows, and the next tile's descriptors (issued before
    // them): newer are, after the first tile, the claim and the previous
    // tile's record stores.
    STAMP(0, __builtin_amdgcn_s_memrealtime());
    if (it_ == 0) vm_wait<0>();
    else vm_wait<1 + NST>();
    STAMP(1, __builtin_amdgcn_s_memrealtime());
#ifdef OO_RX_STAMPS
    if (lane == 0)
      dstamp_slot(P.stamps != nullptr && it_ < 128 ? &P.stamps[((size_t)gwave * 128 + it_) * 16] : nullptr,
                  true);
#endif
    // The claim made at the last tile's staging: the tile after the next
    // one.  (Read here, not in the staging below, where the compiler's wait
    // for it would also wait for the key index loads.  Claiming at the
    // tile's start instead, before those loads, measured 4 % slower on
    // config 3: profiles/r06/ab_win_stage_overlap_c3_c4.log.)
    if (it_ != 0) {
      const uint32_t c = (uint32_t)__builtin_amdgcn_readfirstlane((int)got);
      tnext2 = P.dyn ? 3u * W + g + c : tnext2 + W;
    }
    const DescView dv = desc_view(P, lds_read16(&L.desc[b][lane]), tile, lane);
    // (the window's cell addresses recomputed per tile: hoisted, eight
    // loop-long registers would spill)
    uint32_t wl = lane;
    asm volatile("" : "+v"(wl));
    const Hdr h = parse_headers<OO_RX_GEN_RUNS>(window_of(L.hdr, wl), dv.shift, dv.len, dv.abase);
    STAMP(2, __builtin_amdgcn_s_memrealtime());
    // ---- lookups and the record.  The next tile is staged inside the
    // demux, as soon as the key index's loads are issued and before they
    // are waited for, so the lookup's round trip and the staging's overlap
    // (DESIGN.md §5 round 6): the descriptors of the tile after it into the
    // buffer this tile's came in (read above), its windows into the rows
    // the parse has read, the claim of the tile after that.
    auto stage = [&]() {
      glds<0>(desc_src(P, unit_of(P, tnext2), lane), &L.desc[b][0]);
      const Unit nt = unit_of(P, tnext);
      const DescView dn = desc_view(P, lds_read16(&L.desc[b ^ 1u][lane]), nt, lane);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the parse's LDS reads are done
      const bool short4 = __ballot(dn.span > 64) == 0;
      if (__ballot(dn.span > HB) == 0)  // no frame of the tile has a body
        stage_window<OO_RX_WIN_HDR_AUX>(dn, zero_line(P, nt, lane), L.hdr, lane,
                                        OO_RX_WIN_MASKED && clean && short4);
      else
        stage_window<OO_RX_HDR_AUX>(dn, zero_line(P, nt, lane), L.hdr, lane, false);
      clean = short4;
      claim_tile(P.claim + 32u * g, P.ngroups, lane, got);
    };
    Parsed ps = demux_packet<true, true>(P, h, dv.intf_i, dv.abase, dv.span, dv.shift, lds_occ, stage);

    STAMP(3, __builtin_amdgcn_s_memrealtime());
    STAMP(4, __builtin_amdgcn_s_memrealtime());
#ifdef OO_RX_PAD_VALU  // (experiment: N dependent VALU instructions per tile, nothing else)
    {
#ifdef OO_RX_PADI  // eight independent chains: the issue cost without the latency
      uint32_t pad[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) pad[j] = lane + j;
#pragma unroll
      for (int i = 0; i < OO_RX_PAD_VALU; ++i) asm volatile("v_add_u32 %0, 1, %0" : "+v"(pad[i & 7]));
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" ::"v"(pad[j]));
#else
      uint32_t pad = lane;
#pragma unroll
      for (int i = 0; i < OO_RX_PAD_VALU; ++i) asm volatile("v_add_u32 %0, 1, %0" : "+v"(pad));
      asm volatile("" ::"v"(pad));
#endif
    }
#endif
    const uint32_t reason = ps.r.reason;
    store_records<OO_RX_WIN_REC_DIRECT>(P, tile, ps.r, lane);
    // The pending words of a tile holding frames with a body.
    const bool body = dv.span > HB;
    if (__ballot(body) != 0) {
      const bool wait = (ps.odd_long & 2u) != 0;
      const uint32_t tgt = wait ? body_target(ps.s4, ps.pseudo, (ps.odd_long & 1u) != 0) : PEND_NONE;
      const uint32_t lo = tgt | (ps.r.proto == 6u ? 1u << 16 : 0u) |
                          ((uint32_t)(ps.r.flags & (OO_RX_F_IP6 | OO_RX_F_VLAN)) << 17) |
                          ((uint32_t)ps.r.reason << 24);
      const uint32_t hi = (uint32_t)ps.r.vlan | ((uint32_t)ps.r.ip_paylen << 16);
      if (lane < tile.cnt) P.pend[tile.first + lane] = (uint64_t)lo | ((uint64_t)hi << 32);
      waits = waits || __ballot(wait) != 0;
    }
    if (P.counters != nullptr) cnt += reason_hist(reason, dv.valid, lane);
    STAMP(5, __builtin_amdgcn_s_memrealtime());
    tcur = tnext;
    tnext = tnext2;
  }
  if (P.counters != nullptr && lane < OO_RX_R_COUNT && cnt != 0) atomicAdd(&P.counters[lane], cnt);
  // The body flag, once a wave and after its tiles: every wave storing to
  // the one line per tile serializes the stores, and the tile loop's counted
  // waits would wait for them.
  if (waits && lane == 0) __hip_atomic_store(P.flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(WAVES_W * 64) __attribute__((amdgpu_waves_per_eu(OO_RX_WIN_WPE))) void win_kernel(
    KParams P) {
#ifdef OO_RX_STAMPS
  dstamp_slot(nullptr, true);  // (no phase stamps from this kernel's demux)
#endif
  window_loop(P);
}
#endif  // !OO_RX_SHORT

// ---------------------------------------------------------------------------
// body_kernel: units of up to 64 packets (its own partition, finer at the
// batch's end); per unit the packets whose pending word waits for the body
// are the jobs of the body engine (lockstep slots, as tile_loop), an RB-slot
// ring with nothing else in the wave's memory queue.  A slot's first F
// rounds hold a whole chunk for every lane (F from the slot's smallest job),
// so they take neither the per-lane live/partial tests nor the per-lane
// advance test.
#ifndef OO_RX_BODY_RING
#define OO_RX_BODY_RING 8
#endif
constexpr int RB = OO_RX_BODY_RING;
static_assert(RB % 2 == 0, "the ring is consumed two pieces at a time");
constexpr int WAVES_B = 2;

struct BodyLds {
  uint4 ring[RB][64];
  uint4 desc[2][64];             // descriptors of this unit and the next
  uint32_t pend[2][2][64];       // their pending words (low, high halves)
  uint32_t dbase, gofs, pad0, pad1;
};
static_assert(sizeof(BodyLds) % 16 == 0, "BodyLds is carved from a uint4 array");
constexpr int BODY_U4 = (int)(sizeof(BodyLds) / 16);
constexpr int MTAB_U4 = 17;  // the block's byte masks of a chunk by valid-byte count 0..16
#ifndef OO_RX_BODY_MTAB
#define OO_RX_BODY_MTAB 1  // the sequences engine takes its masks from the table
#endif

// The block's mask table (before any LDS-DMA; all threads, one barrier).
__device__ __forceinline__ const uint4* body_mask_table(uint4* smem_tab) {
  const uint32_t t = threadIdx.x;
  if (t < (uint32_t)MTAB_U4) {
    auto bytes = [](int k) -> uint32_t {
      return k >= 4 ? 0xffffffffu : k <= 0 ? 0u : (1u << (8 * k)) - 1u;
    };
    const int vb = (int)t;
    smem_tab[t] = make_uint4(bytes(vb), bytes(vb - 4), bytes(vb - 8), bytes(vb - 12));
  }
  __syncthreads();
  return smem_tab;
}

// min(v) over the lanes with the same lane & 7 (as max_x8).
__device__ __forceinline__ uint32_t min_x8(uint32_t v) {
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, false));  // row_ror:8
  v = min(v, (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x401f));  // lane ^ 16
  const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);  // lane ^ 32
  return min((uint32_t)p[0], (uint32_t)p[1]);
}

// The rounds of slot js in which every lane reads a whole chunk that is not
// its job's last: its smallest job's (nb - 1) / 8 (0 when a group has none).
// fm: min_x8 of the jobs' chunk counts (lane j: slot j's).
__device__ __forceinline__ uint32_t slot_full(uint32_t fm, uint32_t js) {
  const uint32_t m = js < 8u ? (uint32_t)__builtin_amdgcn_readlane((int)fm, (int)js) : 0u;
  return m != 0 ? (m - 1u) >> 3 : 0u;
}

// The loads of a unit's descriptors and pending words into buffer b (three
// operations).
__device__ __forceinline__ void stage_unit(const KParams& P, const Unit& u, uint32_t lane,
                                           BodyLds& L, uint32_t b) {
  glds<0>(desc_src(P, u, lane), &L.desc[b][0]);
  const uint32_t i = u.first + lane;  // in the padded pend array (n + 64 entries)
  const uint64_t pa = reinterpret_cast<uint64_t>(P.pend) + 8ull * i;
  __builtin_amdgcn_global_load_lds(reinterpret_cast<gptr>(pa), (lptr)(&L.pend[b][0][0]), 4, 0, 0);
  __builtin_amdgcn_global_load_lds(reinterpret_cast<gptr>(pa + 4u), (lptr)(&L.pend[b][1][0]), 4, 0, 0);
}

// The verdicts of one unit: a failing sum turns the record into the drop
// record (only the fields a drop defines), the per-reason counts move.
__device__ __forceinline__ void unit_verdicts(const KParams& P, bool job, uint32_t bsum,
                                              uint32_t plo, uint32_t phi, uint32_t idx) {
  const bool fail = job && res16(bsum) != (plo & 0xffffu);
  if (__ballot(fail) != 0) {
    if (fail) {
      const bool tcp = (plo >> 16) & 1u;
      const uint32_t reason = tcp ? OO_RX_R_TCP_CSUM : OO_RX_R_UDP_CSUM;
      const uint4 r0 = make_uint4(reason | (((plo >> 17) & 3u) << 8) | ((tcp ? 6u : 17u) << 24),
                                  phi & 0xffffu, phi >> 16, 0u);
      const uint4 r1 = make_uint4(0u, 0u, 0xffffffffu, 0u);
      uint4* const o = reinterpret_cast<uint4*>(P.out) + 2ull * idx;
      o[0] = r0;
      o[1] = r1;
      if (P.counters != nullptr) {  // (rare: one frame in a hundred)
        atomicAdd(&P.counters[(plo >> 24) & (OO_RX_R_COUNT - 1)], 0xffffffffu);
        atomicAdd(&P.counters[reason], 1u);
      }
    }
  }
}

#if OO_RX_GSEQ
// One unit as the continuous stream sees it: its jobs and what its verdicts
// need.
struct BUnit {
  Jobs J;
  uint32_t myslot, plo, phi, idx;
  bool job;
  uint64_t zero;
  uint32_t T;  // rounds, a multiple of RB (0: no job)
};
__device__ __forceinline__ BUnit bunit_read(const KParams& P, BodyLds& L, uint32_t b, uint32_t t,
                                            uint32_t lane) {
  BUnit U;
  const Unit unit = unit_of(P, t);
  const DescView dv = desc_view(P, lds_read16(&L.desc[b][lane]), unit, lane);
  U.plo = lds_read4(&L.pend[b][0][lane]);
  U.phi = lds_read4(&L.pend[b][1][lane]);
  U.idx = dv.idx;
  U.zero = zero_line(P, unit, lane);
  U.job = dv.valid && dv.span > HB && (U.plo & 0xffffu) != PEND_NONE;
  U.J = jobs_setup(dv.abase, U.job ? dv.span : 0, lane, U.myslot);
  U.T = (U.J.T + RB - 1) / RB * RB;
  return U;
}

// body_loop with per-group job sequences and one continuous stream: the
// ring is not drained at a unit's end -- its last turn issues the first
// rounds of the next unit, whose jobs were set up at the unit's start -- so
// a wave pays the memory latency once per run of units with bodies, not
// once per unit.  Each iteration reads the next unit's descriptors and
// pending words (staged one unit earlier), stages the unit after it into the
// buffer the current unit was read from, and claims the one after that.
__device__ __forceinline__ void body_loop(const KParams& P) {
  __shared__ __attribute__((aligned(16))) uint4 smem[WAVES_B * BODY_U4 + MTAB_U4];
  const int wave = (int)(threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63u;
  BodyLds& L = reinterpret_cast<BodyLds*>(smem)[wave];
  const uint4* const mtab = OO_RX_BODY_MTAB ? body_mask_table(smem + WAVES_B * BODY_U4) : nullptr;
  const uint32_t gwave = sreg(blockIdx.x * WAVES_B + wave);
  const uint32_t W = gridDim.x * WAVES_B;
  // No frame of the batch waits for its body: nothing to do.
  if (__hip_atomic_load(P.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) return;
  if (gwave >= P.ntiles) return;
  uint32_t tcur = gwave, tnext = gwave + W, tnext2 = gwave + 2u * W, got = 0;
  if (lane == 0) {
    const uint32_t g = group_of(P, gwave);
    lds_write4(&L.dbase, 3u * W + g);
    lds_write4(&L.gofs, 32u * g);
  }
  stage_unit(P, unit_of(P, tcur), lane, L, 0);
  stage_unit(P, unit_of(P, tnext), lane, L, 1);
  vm_wait<0>();

  BUnit C = bunit_read(P, L, 0, tcur, lane);
  IssueCursor ci;
  ConsumeCursor cc;
  if (C.T != 0) {
    issue_slot(ci, C.J, 0, lane, C.zero);
#pragma unroll
    for (int u = 0; u < RB; ++u) issue_round(ci, C.J, C.zero, &L.ring[u][0], lane);
  }
  uint32_t b = 0;
  // Vector-memory operations issued after the last staging when the
  // iteration that issued it waited for none of them (a unit without jobs):
  // its claim, and the next unit's first rounds if it primed them.
  int unwaited = 0;
  for (uint32_t it_ = 0; tcur < P.ntiles; b ^= 1u, ++it_) {
    // ---- the next unit (staged in buffer b ^ 1 one iteration ago: landed
    // once that iteration's waits passed rounds issued after it), then the
    // unit after it staged into buffer b (read one iteration ago) and the one
    // after that claimed: all older than the rounds the waits below count.
    if (unwaited != 0) vm_wait_n(unwaited - 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const BUnit N = bunit_read(P, L, b ^ 1u, tnext, lane);
    if (it_ != 0) {
      const uint32_t c = (uint32_t)__builtin_amdgcn_readfirstlane((int)got);
      tnext2 = P.dyn ? sreg(lds_read4(&L.dbase)) + c : tnext2 + W;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    stage_unit(P, unit_of(P, tnext2), lane, L, b);
    claim_tile(P.claim + sreg(lds_read4(&L.gofs)), P.ngroups, lane, got);

    uint32_t bsum = 0;
    unwaited = C.T != 0 ? 0 : 2;  // (the claim; +RB below)
    if (C.T != 0) {
      IssueCursor ni;  // the next unit's first rounds go out in this unit's last turn
      const bool carry = N.T != 0;
      if (carry) issue_slot(ni, N.J, 0, lane, N.zero);
      consume_start(cc, C.J, lane, mtab);
      for (uint32_t k0 = 0; k0 < C.T; k0 += RB) {
        const bool last = k0 + RB == C.T;
#pragma unroll
        for (int u = 0; u < RB; u += 2) {
          if (last && !carry) vm_wait_n(RB - 2 - u);
          else vm_wait<RB - 2>();
          uint4 v0, v1;
          lds_read16x2(&L.ring[u][lane], &L.ring[u + 1][lane], v0, v1);
          consume_round(cc, C.J, v0, lane, mtab);
          consume_round(cc, C.J, v1, lane, mtab);
          if (!last) {
            issue_round(ci, C.J, C.zero, &L.ring[u][0], lane);
            issue_round(ci, C.J, C.zero, &L.ring[u + 1][0], lane);
          } else if (carry) {
            issue_round(ni, N.J, N.zero, &L.ring[u][0], lane);
            issue_round(ni, N.J, N.zero, &L.ring[u + 1][0], lane);
          }
        }
      }
      bsum = lane_get(cc.bs, C.myslot);
      if (carry) ci = ni;
    } else if (N.T != 0) {  // nothing here: start the next unit's stream
      issue_slot(ci, N.J, 0, lane, N.zero);
#pragma unroll
      for (int u = 0; u < RB; ++u) issue_round(ci, N.J, N.zero, &L.ring[u][0], lane);
      unwaited += RB;
    }
    unit_verdicts(P, C.job, bsum, C.plo, C.phi, C.idx);
    C = N;
    tcur = tnext;
    tnext = tnext2;
  }
}
#else
__device__ __forceinline__ void body_loop(const KParams& P) {
  __shared__ __attribute__((aligned(16))) uint4 smem[WAVES_B * BODY_U4];
  const int wave = (int)(threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63u;
  BodyLds& L = reinterpret_cast<BodyLds*>(smem)[wave];
  const uint32_t gwave = sreg(blockIdx.x * WAVES_B + wave);
  const uint32_t W = gridDim.x * WAVES_B;
  // No frame of the batch waits for its body: nothing to do.
  if (__hip_atomic_load(P.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) return;
  if (gwave >= P.ntiles) return;
  uint32_t tcur = gwave, tnext = gwave + W, tnext2 = gwave + 2u * W, got = 0;
  if (lane == 0) {
    const uint32_t g = group_of(P, gwave);
    lds_write4(&L.dbase, 3u * W + g);
    lds_write4(&L.gofs, 32u * g);
  }
  stage_unit(P, unit_of(P, tcur), lane, L, 0);
  stage_unit(P, unit_of(P, tnext), lane, L, 1);
  vm_wait<0>();

  uint32_t b = 0;
  for (uint32_t it_ = 0; tcur < P.ntiles; b ^= 1u, ++it_) {
    const Unit unit = unit_of(P, tcur);
    const DescView dv = desc_view(P, lds_read16(&L.desc[b][lane]), unit, lane);
    const uint32_t plo = lds_read4(&L.pend[b][0][lane]);
    const uint32_t phi = lds_read4(&L.pend[b][1][lane]);
    const uint64_t zero = zero_line(P, unit, lane);
    // Jobs: the frames with a body whose verdict waits for it.
    const uint32_t tgt = plo & 0xffffu;
    const bool job = dv.valid && dv.span > HB && tgt != PEND_NONE;
    uint32_t myslot;
    const Jobs J = jobs_setup(dv.abase, job ? dv.span : 0, lane, myslot);
    const uint32_t fm = min_x8(J.nb);

    // ---- stage the unit after next (into this unit's buffers, now read)
    // and claim the one after that: older than this unit's rounds, so the
    // ring's waits need not count them.
    if (it_ != 0) {
      const uint32_t c = (uint32_t)__builtin_amdgcn_readfirstlane((int)got);
      tnext2 = P.dyn ? sreg(lds_read4(&L.dbase)) + c : tnext2 + W;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    stage_unit(P, unit_of(P, tnext2), lane, L, b);
    claim_tile(P.claim + sreg(lds_read4(&L.gofs)), P.ngroups, lane, got);

    const uint32_t T = (J.T + RB - 1) / RB * RB;
    uint32_t bsum = 0;
    if (T != 0) {
      IssueCursor ci;
      issue_slot(ci, J, 0, lane, zero);
      // issue side
      uint32_t fi = slot_full(fm, 0);
      auto issue = [&](void* slot) {
        glds<OO_RX_BODY_AUX>(ci.a, slot);
        if (ci.rnd + 1u < fi) ci.a += 128u;  // every lane reads on (scalar test)
        else ci.a += ci.rnd < ci.adv ? 128u : 0u;
        if (++ci.rnd == ci.R) {
          issue_slot(ci, J, ci.js + 1, lane, zero);
          fi = slot_full(fm, ci.js);
        }
      };
#pragma unroll
      for (int u = 0; u < RB; ++u) issue(&L.ring[u][0]);
      // consume side
      ConsumeCursor cc;
      consume_start(cc, J, lane);
      uint32_t fc = slot_full(fm, 0);
      auto consume = [&](const uint4& v) {
        if (cc.rnd < fc) {  // every lane: a whole chunk, not its last
          uint32_t a = dot(v.x, 0x00010001u, cc.acc);
          uint32_t b2 = dot(v.y, 0x00010001u, 0u);
          a = dot(v.z, 0x00010001u, a);
          b2 = dot(v.w, 0x00010001u, b2);
          cc.acc = a + b2;
          ++cc.rnd;
        } else {
          consume_round(cc, J, v, lane);  // (it moves to the next slot itself)
          if (cc.rnd == 0) fc = slot_full(fm, cc.js);
        }
      };
      for (uint32_t k0 = 0; k0 < T; k0 += RB) {
        const bool last = k0 + RB == T;
#pragma unroll
        for (int u = 0; u < RB; u += 2) {
          if (last) vm_wait_n(RB - 2 - u);
          else vm_wait<RB - 2>();
          uint4 v0, v1;
          lds_read16x2(&L.ring[u][lane], &L.ring[u + 1][lane], v0, v1);
          consume(v0);
          consume(v1);
          if (!last) {
            issue(&L.ring[u][0]);
            issue(&L.ring[u + 1][0]);
          }
        }
      }
      bsum = lane_get(cc.bs, myslot);
    }

    unit_verdicts(P, job, bsum, plo, phi, dv.idx);
    tcur = tnext;
    tnext = tnext2;
  }
}

#endif  // OO_RX_GSEQ

__global__ __launch_bounds__(WAVES_B * 64) void body_kernel(KParams P) { body_loop(P); }
#endif  // !OO_RX_POLL

}  // namespace oo_rx

#if defined(OO_RX_POLL)
extern "C" int oo_rx_blocks_per_cu_poll(void) {
  int b = 0;
  const hipError_t e =
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, oo_rx_poll::rx_kernel, oo_rx_poll::WAVES * 64, 0);
  return e == hipSuccess ? b : 0;
}

// Launch one poll-sized RX batch on `stream` (oo_rx_poll::rx_kernel).
extern "C" int oo_rx_launch_poll(const oo_rx::PollArgs* A, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(oo_rx_poll::rx_kernel, dim3(grid), dim3(oo_rx_poll::WAVES * 64), 0, stream, *A);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

#elif defined(OO_RX_SHORT)
// Resident blocks per CU of the short-frame rx_kernel.
extern "C" int oo_rx_blocks_per_cu_short(void) {
  int b = 0;
  const hipError_t e =
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, oo_rx_short::rx_kernel, oo_rx_short::WAVES * 64, 0);
  return e == hipSuccess ? b : 0;
}

// Launch one RX batch of short frames on `stream`.
extern "C" int oo_rx_launch_short(const oo_rx::KParams* P, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(oo_rx_short::rx_kernel, dim3(grid), dim3(oo_rx_short::WAVES * 64), 0, stream, *P);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// The split transform's body_kernel with per-group job sequences (mixed
// frame sizes).
extern "C" int oo_rx_body_blocks_per_cu_gseq(void) {
  int b = 0;
  const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, oo_rx_short::body_kernel,
                                                                     oo_rx_short::WAVES_B * 64, 0);
  return e == hipSuccess ? b : 0;
}
extern "C" int oo_rx_launch_body_gseq(const oo_rx::KParams* P, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(oo_rx_short::body_kernel, dim3(grid), dim3(oo_rx_short::WAVES_B * 64), 0, stream, *P);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
#else
// Resident blocks per CU (sizes the persistent grid).
extern "C" int oo_rx_blocks_per_cu(void) {
  int b = 0;
  const hipError_t e =
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, oo_rx::rx_kernel, oo_rx::WAVES * 64, 0);
  return e == hipSuccess ? b : 0;
}

// Tile-processing waves per block.
extern "C" int oo_rx_waves_per_block(void) { return oo_rx::WAVES; }

// Launch one TX checksum fill batch on `stream` (rx_kernel's grid).
extern "C" int oo_tx_launch(const oo_rx::KParams* P, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(oo_rx::tx_kernel, dim3(grid), dim3(oo_rx::WAVES * 64), 0, stream, *P);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Launch one RX batch on `stream`.
extern "C" int oo_rx_launch(const oo_rx::KParams* P, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(oo_rx::rx_kernel, dim3(grid), dim3(oo_rx::WAVES * 64), 0, stream, *P);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// The split transform's two kernels: resident blocks per CU, waves per
// block, launches.
extern "C" int oo_rx_win_blocks_per_cu(void) {
  int b = 0;
  const hipError_t e =
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, oo_rx::win_kernel, oo_rx::WAVES_W * 64, 0);
  return e == hipSuccess ? b : 0;
}
extern "C" int oo_rx_body_blocks_per_cu(void) {
  int b = 0;
  const hipError_t e =
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, oo_rx::body_kernel, oo_rx::WAVES_B * 64, 0);
  return e == hipSuccess ? b : 0;
}
extern "C" int oo_rx_win_waves_per_block(void) { return oo_rx::WAVES_W; }
extern "C" int oo_rx_body_waves_per_block(void) { return oo_rx::WAVES_B; }
extern "C" int oo_rx_launch_win(const oo_rx::KParams* P, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(oo_rx::win_kernel, dim3(grid), dim3(oo_rx::WAVES_W * 64), 0, stream, *P);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
extern "C" int oo_rx_launch_body(const oo_rx::KParams* P, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(oo_rx::body_kernel, dim3(grid), dim3(oo_rx::WAVES_B * 64), 0, stream, *P);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
#endif  // OO_RX_SHORT
