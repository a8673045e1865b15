// SPDX-License-Identifier: BSD-2-Clause
//
// oo_rx_kernel.hip -- gfx950 (MI355X / CDNA4) kernel for Onload's software
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
// One kernel, rx_kernel (DESIGN.md "Kernel").  Each wave owns tiles of 64
// packets and strides over them; per tile:
//   1. descriptors: one coalesced 16-B load per lane (next tile's prefetched);
//   2. header staging: the first 128 window bytes of the 64 frames, coalesced
//      16-B loads (8 lanes x 16 B per frame per instruction) written
//      transposed into LDS as [chunk][packet] cells;
//   3. per lane (one packet per lane): VLAN, L3/L4 gates, pseudo-header,
//      IPv4 header sum and the L4 sum inside the window, and every header
//      field the rest of the path needs, read out of LDS into registers;
//   4. the tile's long L4 regions (past the window) are concatenated into
//      one flat list of 16-B chunks and streamed in full 1-KiB pieces by
//      LDS-DMA (global_load_lds_dwordx4, nontemporal) into an 8-piece ring
//      that reuses the staging LDS; each piece is reduced by a segmented
//      wave scan (DPP) and per-packet partial sums land in LDS;
//   5. per lane: verdict, handle_rx_pkt's frag/options/TCP-scattered tests,
//      the 2 or 3 filter-table lookup stages (IPv4 first probes issued before
//      the stream so their latency hides under it), and the 32-B record.
//   Per-reason counters accumulate in LDS and are flushed once per block.
//
// The verdict uses the mod-0xffff residue of the exact word sum; see
// oracle/rx_oracle.c for why that equals the reference's folded-complement
// test (and why it may be summed in any grouping).  No MFMA: integer
// reduction + table probes, HBM-bound.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "oo_rx_device.h"

namespace oo_rx {

typedef unsigned short v2u16 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Tuning knobs (compile-time; `make variants` builds sweeps of them).
#ifndef OO_RX_WAVES
#define OO_RX_WAVES 2
#endif
#ifndef OO_RX_SP
#define OO_RX_SP 4
#endif
#ifndef OO_RX_WPE
#define OO_RX_WPE 4  // amdgpu_waves_per_eu target, 0 = compiler's choice
#endif

constexpr int WAVES = OO_RX_WAVES;   // waves per block
constexpr int HC = 8;                // staged header chunks per packet
constexpr int HB = HC * 16;          // staged window bytes per packet
constexpr int ROWB = 64 * 16 + 16;   // one staged chunk of all 64 packets (+pad)
constexpr int SP = OO_RX_SP;
static_assert(SP % 4 == 0, "ku packs 4 pieces per register");                // 1-KiB stream pieces per register buffer


// Filter-table entry states (netif_table.c:34-42).
constexpr uint32_t ST_MASK = 0xc0000000u;
constexpr uint32_t ID_MASK = 0x3fffffffu;
constexpr uint32_t ST_PREFERRED = 0x00000000u;
constexpr uint32_t ST_EMPTY = 0x80000000u;
constexpr uint32_t ST_TOMBSTONE = 0xc0000000u;
constexpr int ID6_EMPTY = -2;
constexpr uint32_t PENDING = 0xffu;

typedef const __attribute__((address_space(1))) u32x4* gptr_u32x4;

// Nontemporal 16-byte load from global memory.  The explicit global address
// space matters: a pointer rebuilt from integers would otherwise compile to
// a flat load, which also counts on lgkmcnt and so stalls every LDS wait
// behind the HBM stream.
__device__ __forceinline__ uint4 ld_stream(uint64_t addr) {
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<gptr_u32x4>(addr));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint4 ld_stream(const void* p) {
  return ld_stream(reinterpret_cast<uint64_t>(p));
}

__device__ __forceinline__ bool occupied(uint32_t st) {
  return ((~st) & ST_EMPTY & ST_TOMBSTONE) != 0;
}

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// hash.h:84-93 / 165-173; network-order values in host integers.
__device__ __forceinline__ uint32_t hash3(uint32_t la, uint32_t lp, uint32_t ra,
                                          uint32_t rp, uint32_t proto) {
  uint32_t h = __builtin_bswap32(ra) ^ la ^ ((rp << 16) | lp) ^ proto;
  h ^= h >> 16;
  h ^= h >> 8;
  return h;
}
__device__ __forceinline__ uint32_t hash2(uint32_t la, uint32_t lp, uint32_t ra,
                                          uint32_t rp, uint32_t proto) {
  return ((la ^ ra) ^ ((lp << 16) | rp) ^ proto) | 1u;
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

// Inclusive sum over a 16-lane DPP row; lane 15 of the row holds the total.
__device__ __forceinline__ uint32_t row_sum16(uint32_t v) {
  v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, true);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, true);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, true);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, true);  // row_shr:8
  return v;
}

// ---------------------------------------------------------------------------
// Demux: one lookup stage walked to its end (every match counted).

struct Match {
  int32_t first;
  uint32_t n;
};

__device__ __forceinline__ bool bind2dev_ok(const KParams& P, const oo_gpu_rx_sock& s,
                                            int intf_i, int vlan) {
  if (!(s.flags & OO_GPU_RX_SOCK_BIND2DEV)) return true;
  const uint32_t hw =
      (intf_i >= 0 && intf_i < OO_GPU_RX_MAX_INTF) ? P.hwport[intf_i] : 0xffu;
  return hw < 64 && (s.bind2dev_hwports & (1ull << hw)) != 0 && s.bind2dev_vlan == vlan;
}

__device__ __forceinline__ oo_gpu_rx_sock load_sock(const KParams& P, uint32_t id) {
  const uint4* p = reinterpret_cast<const uint4*>(P.socks + id);
  oo_gpu_rx_sock s;
  uint4* d = reinterpret_cast<uint4*>(&s);
  d[0] = p[0];
  d[1] = p[1];
  d[2] = p[2];
  return s;
}

// ci_netif_filter_for_each_match (netif_table.c:234-319), starting from the
// already-loaded entry e at slot h1 = hash1.
__device__ Match walk4(const KParams& P, uint32_t la, uint32_t lp, uint32_t ra, uint32_t rp,
                       uint32_t proto, int intf_i, int vlan, uint32_t h1, uint2 e) {
  Match m = {-1, 0};
  const uint32_t mask = P.ip4_mask;
  const uint32_t first = h1;
  const uint32_t h2 = hash2(la, lp, ra, rp, proto);
  bool check_lport = false;
  for (uint32_t guard = 0; guard <= mask; ++guard) {
    const uint32_t st = e.x & ST_MASK;
    if (check_lport ? occupied(st) : st == ST_PREFERRED) {
      const uint32_t id = e.x & ID_MASK;
      if (e.y == la && id < P.max_socks) {
        const oo_gpu_rx_sock s = load_sock(P, id);
        bool ok = s.raddr_be32 == ra && s.rport_be16 == rp && s.protocol == proto;
        if (check_lport) ok = ok && (P.ip4_ext[h1].y & 0xffffu) == lp;
        if (ok && bind2dev_ok(P, s, intf_i, vlan)) {
          if (m.n == 0) m.first = (int32_t)id;
          ++m.n;
        }
      }
    }
    if (st == ST_EMPTY) break;
    h1 = (h1 + h2) & mask;
    if (h1 == first) break;
    e = P.ip4[h1];
    check_lport = true;
  }
  return m;
}

// ci_netif_filter_for_each_match_ip6 (netif_table_ip6.c:110-189), starting
// from the already-loaded entry e at slot h1.
__device__ Match walk6(const KParams& P, const uint32_t la[4], uint32_t lp, const uint32_t ra[4],
                       bool ra_null, uint32_t rp, uint32_t proto, int intf_i, int vlan,
                       uint32_t h1, Ip6Entry e) {
  Match m = {-1, 0};
  const uint32_t mask = P.ip6_mask;
  const uint32_t lx = la[0] ^ la[1] ^ la[2] ^ la[3];
  const uint32_t rx = ra_null ? 0u : (ra[0] ^ ra[1] ^ ra[2] ^ ra[3]);
  const uint32_t first = h1;
  const uint32_t h2 = hash2(lx, lp, rx, rp, proto);
  for (uint32_t guard = 0; guard <= mask; ++guard) {
    if (e.id >= 0) {
      if ((uint32_t)e.id < P.max_socks && e.laddr[0] == la[0] && e.laddr[1] == la[1] &&
          e.laddr[2] == la[2] && e.laddr[3] == la[3]) {
        const oo_gpu_rx_sock s = load_sock(P, (uint32_t)e.id);
        bool ok = s.lport_be16 == lp && s.protocol == proto;
        if (ok) {
          if (ra_null) {
            ok = !(s.flags & OO_GPU_RX_SOCK_CONNECTED);
          } else {
            uint32_t r6[4];
            __builtin_memcpy(r6, s.raddr6, 16);
            ok = r6[0] == ra[0] && r6[1] == ra[1] && r6[2] == ra[2] && r6[3] == ra[3] &&
                 s.rport_be16 == rp;
          }
        }
        if (ok && bind2dev_ok(P, s, intf_i, vlan)) {
          if (m.n == 0) m.first = e.id;
          ++m.n;
        }
      }
    } else if (e.id == ID6_EMPTY) {
      break;
    }
    h1 = (h1 + h2) & mask;
    if (h1 == first) break;
    e = P.ip6[h1];
  }
  return m;
}

__device__ __forceinline__ uint32_t opaque(uint32_t x) {
  asm volatile("" : "+v"(x));
  return x;
}

// Inclusive max over all 64 lanes (same DPP pattern as wave_scan).
__device__ __forceinline__ uint32_t wave_max_scan(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, true));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, true));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, true));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, true));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false));
  return v;
}

// Inclusive sum over all 64 lanes (DPP row shifts, then row broadcasts).
__device__ __forceinline__ uint32_t wave_scan(uint32_t v) {
  v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, true);   // row_shr:1
  v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, true);   // row_shr:2
  v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, true);   // row_shr:4
  v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, true);   // row_shr:8
  v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}

// ---------------------------------------------------------------------------

#if OO_RX_WPE > 0
#define OO_RX_KATTR __attribute__((amdgpu_waves_per_eu(OO_RX_WPE)))
#else
#define OO_RX_KATTR
#endif

__global__ __launch_bounds__(WAVES * 64) OO_RX_KATTR void rx_kernel(KParams P) {
  __shared__ __attribute__((aligned(16))) uint8_t hdrs[WAVES][HC][ROWB];  // [chunk][packet] cells
  __shared__ __attribute__((aligned(16))) uint4 jobs[WAVES][64];  // {VB lo, VB hi, first chunk, end}
  __shared__ __attribute__((aligned(16))) uint8_t kmaps[WAVES][SP * 64];  // chunk -> packet marks
  __shared__ uint32_t gmarks[WAVES][2][64];  // running sum before / at each packet's run
  __shared__ uint32_t ctr[OO_RX_R_COUNT];

  const int wave = (int)(threadIdx.x >> 6);
  const int lane = (int)(threadIdx.x & 63);
  uint8_t (&hdr)[HC][ROWB] = hdrs[wave];
  uint4* job = jobs[wave];
  uint8_t* kmap = kmaps[wave];
  uint32_t* g_start = gmarks[wave][0];
  uint32_t* g_end = gmarks[wave][1];
  if (threadIdx.x < OO_RX_R_COUNT) ctr[threadIdx.x] = 0;
  __syncthreads();

  const uint32_t ntiles = (P.n + 63) / 64;
  const uint32_t stride = gridDim.x * WAVES;
  uint32_t tile = blockIdx.x * WAVES + wave;
  uint4 dnext = make_uint4(0, 0, 0, 0);
  if (tile < ntiles && tile * 64 + lane < P.n)
    dnext = ld_stream(reinterpret_cast<const uint4*>(P.desc) + tile * 64 + lane);

  for (; tile < ntiles; tile += stride) {
    // ---- 1. descriptor (prefetched), and the next tile's
    const uint32_t idx = tile * 64 + (uint32_t)lane;
    const bool valid = idx < P.n;
    const uint4 d = dnext;
    {
      const uint32_t nidx = (tile + stride) * 64 + (uint32_t)lane;
      dnext = make_uint4(0, 0, 0, 0);
      if (tile + stride < ntiles && nidx < P.n)
        dnext = ld_stream(reinterpret_cast<const uint4*>(P.desc) + nidx);
    }
    const uint64_t off = (uint64_t)d.x | ((uint64_t)d.y << 32);
    int len = (int)(d.z & 0xffffu);
    const int intf_i = (int)(int16_t)(d.z >> 16);
    const bool inb = valid && off + (uint64_t)len <= P.frames_bytes;
    if (!inb) len = 0;  // a descriptor outside the buffer is an empty frame
    const uint64_t base = reinterpret_cast<uint64_t>(P.frames) + (inb ? off : 0);
    const int shift = (int)(base & 15u);
    const uint64_t abase = base - (uint64_t)shift;
    const int span = inb ? shift + len : 0;

    // ---- 2. stage the first HB window bytes of all 64 frames, transposed.
    uint4 stg[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int f = kk * 8 + (lane >> 3);
      const int c = lane & 7;
      const uint32_t ablo = (uint32_t)__shfl((int)(uint32_t)abase, f, 64);
      const uint32_t abhi = (uint32_t)__shfl((int)(uint32_t)(abase >> 32), f, 64);
      const int sp = __shfl(span, f, 64);
      // Unconditional (cells past the frame read the descriptor array, which
      // is always mapped) so all eight loads are in flight together.
      const uint64_t src = c * 16 < sp ? (((uint64_t)abhi << 32) | ablo) + (uint64_t)c * 16
                                       : reinterpret_cast<uint64_t>(P.desc);
      stg[kk] = ld_stream(src);
    }
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int f = kk * 8 + (lane >> 3);
      *reinterpret_cast<uint4*>(&hdr[lane & 7][f * 16]) = stg[kk];
    }
    wave_sync_lds();

    const uint8_t* my = &hdr[0][lane * 16];
    // Header byte j (j >= 0); bytes at or beyond the frame length read 0.
    auto B = [&](int j) -> uint32_t {
      int w = shift + j;
      w = w < HB ? w : HB - 1;
      const uint32_t v = my[(w >> 4) * ROWB + (w & 15)];
      return j < len ? v : 0u;
    };
    auto BE16 = [&](int j) -> uint32_t { return (B(j) << 8) | B(j + 1); };
    auto N16 = [&](int j) -> uint32_t { return B(j) | (B(j + 1) << 8); };
    auto N32 = [&](int j) -> uint32_t { return N16(j) | (N16(j + 2) << 16); };

    // ---- 3. parse (per lane)
    uint8_t flags = 0;
    int pre_l3 = 14, vlan = 0;
    if (BE16(12) == 0x8100u) {  // ci_parse_rx_vlan (netif_event.c:116-132)
      pre_l3 = 18;
      vlan = (int)(BE16(14) & 0xfffu);
      flags |= OO_RX_F_VLAN;
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
        flags |= OO_RX_F_IP6;
        ip_paylen = (int)BE16(l3 + 4);
        proto = B(l3 + 6);
        if (ip_paylen <= 0 || len < pre_l3 + 40 + ip_paylen) reason = OO_RX_R_IP6_LEN;
        l4 = l3 + 40;
      } else {
        reason = OO_RX_R_NOT_IP;  // :1078
      }
    }

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

    // Sums over the staged window: IPv4 header [S3,E3), L4 head [S4,min(E4,HB)).
    const bool need_ip = reason == PENDING && !is6;
    const int S3 = shift + l3, E3 = need_ip ? shift + l3 + ihl4 : S3;
    const int S4 = shift + l4, E4 = need_l4 ? shift + l4 + l4_len : S4;
    const int E4h = E4 < HB ? E4 : HB;
    uint32_t s3 = 0, s4 = 0;
    if (need_ip || need_l4) {
#pragma unroll
      for (int k = 0; k < HC; ++k) {
        const uint4 v = *reinterpret_cast<const uint4*>(my + k * ROWB);
        if (k * 16 < E3) s3 += chunk_sum(v, k * 16, S3, E3);
        if (k * 16 < E4h) s4 += chunk_sum(v, k * 16, S4, E4h);
      }
    }
    if (reason == PENDING && need_ip) {
      // IHL != 0 makes the word sum non-zero: fold == 0xffff <=> valid.
      if (ihl4 == 0 || fold16(s3) != 0xffffu) reason = OO_RX_R_IP4_CSUM;
    }
    if (reason == PENDING && l4_gate != PENDING) reason = l4_gate;

    // L4 verdict now when the region ends inside the window; otherwise it
    // waits for the stream (step 5) and the record below is speculative.
    const bool longl4 = reason == PENDING && need_l4 && E4 > HB;
    if (reason == PENDING && need_l4 && !longl4) {
      uint32_t f = fold16(s4);
      if (shift & 1) f = swap16(f);  // RFC 1071 byte-order swap
      if (fold16(f + pseudo) != 0xffffu)
        reason = proto == 6u ? OO_RX_R_TCP_CSUM : OO_RX_R_UDP_CSUM;
    }

    // ---- 4. handle_rx_pkt, demux, record (per lane; netif_event.c:250-451).
    oo_gpu_rx_result r;
    r.reason = 0; r.flags = 0; r.stage = 0; r.proto = 0; r.vlan = (uint16_t)vlan;
    r.l4_off = 0; r.ip_paylen = 0; r.sport_be = 0; r.dport_be = 0; r.nmatch = 0;
    r.saddr_be = 0; r.daddr_be = 0; r.sock = -1; r.hash3 = 0;
    if (l3ok) {
      r.proto = (uint8_t)proto;
      r.ip_paylen = (uint16_t)ip_paylen;
    }
    if (reason == PENDING) {
      flags |= OO_RX_F_CSUM_OK;
      r.l4_off = (uint16_t)l4;
      const uint32_t sport = N16(l4), dport = N16(l4 + 2);
      r.sport_be = (uint16_t)sport;
      r.dport_be = (uint16_t)dport;
      uint32_t a6s[4], a6d[4];
      if (is6) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          a6s[i] = N32(l3 + 8 + 4 * i);
          a6d[i] = N32(l3 + 24 + 4 * i);
        }
        r.saddr_be = a6s[0] ^ a6s[1] ^ a6s[2] ^ a6s[3];
        r.daddr_be = a6d[0] ^ a6d[1] ^ a6d[2] ^ a6d[3];
      } else {
        r.saddr_be = N32(l3 + 12);
        r.daddr_be = N32(l3 + 16);
        const uint32_t frag = BE16(l3 + 6);
        if ((frag & 0x3fffu) != 0 || ip_len > len - pre_l3) {
          reason = OO_RX_R_IP4_FRAG;  // :293-295
        } else if (ihl4 > 20) {
          // ci_ip_options_parse (netif_event.c:135-185), signed-char lengths.
          int o = l3 + 20;
          const int end = l3 + ihl4;
          bool err = false;
          while (B(o) != 0u && o < end && !err) {
            const uint32_t kind = B(o);
            if (kind == 1u) {
              ++o;
            } else if (kind == 7u || kind == 68u || kind == 130u || kind == 136u) {
              const int l = (int)(int8_t)(uint8_t)B(o + 1);
              if (l < 4 || l > end - o) err = true;
              else o += l;
            } else {
              err = true;
            }
          }
          if (err) reason = OO_RX_R_IP4_OPTS_BAD;
        }
        if (reason == PENDING && proto == 6u && frag != 0x4000u && frag != 0u)
          reason = OO_RX_R_TCP_SCATTERED;  // tcp_rx.c:4696-4699
      }

      if (reason == PENDING) {
        // Demux stages in reference order (udp_rx.c:271-306,
        // tcp_rx.c:4786-4835); the first stage with a match decides.  The
        // first probe of every stage is loaded up front.
        r.hash3 = hash3(r.daddr_be, dport, r.saddr_be, sport, proto);
        if (proto == 17u) {
          // ci_udp_rx_deliver's multi-destination test reads the IPv4 view
          // of the L3 header (udp_rx.c:157-159): bytes 16..19.
          const uint32_t dd = N32(l3 + 16);
          if ((dd & 0xf0u) == 0xe0u || dd == 0xffffffffu) flags |= OO_RX_F_MCAST;
        }
        const int nst = proto == 6u ? 3 : 2;
        Match m = {-1, 0};
        int stage = 0;
        if (is6) {
          const uint32_t zero[4] = {0, 0, 0, 0};
          const uint32_t dx = r.daddr_be, sx = r.saddr_be;
          const uint32_t h1_0 = hash3(dx, dport, sx, sport, proto) & P.ip6_mask;
          const uint32_t h1_1 = hash3(dx, dport, 0u, 0u, proto) & P.ip6_mask;
          const uint32_t h1_2 = hash3(0u, dport, 0u, 0u, proto) & P.ip6_mask;
          m = walk6(P, a6d, dport, a6s, false, sport, proto, intf_i, vlan, h1_0, P.ip6[h1_0]);
          stage = 1;
          if (m.n == 0) {
            m = walk6(P, a6d, dport, zero, true, 0u, proto, intf_i, vlan, h1_1, P.ip6[h1_1]);
            stage = 2;
          }
          if (m.n == 0 && nst == 3) {
            m = walk6(P, zero, dport, zero, true, 0u, proto, intf_i, vlan, h1_2, P.ip6[h1_2]);
            stage = 3;
          }
        } else {
          const uint32_t da = r.daddr_be, sa = r.saddr_be;
          const uint32_t h1_0 = hash3(da, dport, sa, sport, proto) & P.ip4_mask;
          const uint32_t h1_1 = hash3(da, dport, 0u, 0u, proto) & P.ip4_mask;
          const uint32_t h1_2 = hash3(0u, dport, 0u, 0u, proto) & P.ip4_mask;
          const uint2 e0 = P.ip4[h1_0];
          const uint2 e1 = P.ip4[h1_1];
          uint2 e2 = e1;
          if (nst == 3) e2 = P.ip4[h1_2];
          m = walk4(P, da, dport, sa, sport, proto, intf_i, vlan, h1_0, e0);
          stage = 1;
          if (m.n == 0) {
            m = walk4(P, da, dport, 0u, 0u, proto, intf_i, vlan, h1_1, e1);
            stage = 2;
          }
          if (m.n == 0 && nst == 3) {
            m = walk4(P, 0u, dport, 0u, 0u, proto, intf_i, vlan, h1_2, e2);
            stage = 3;
          }
        }
        reason = OO_RX_R_NO_MATCH;
        if (m.n) {
          reason = OO_RX_R_DELIVER;
          r.stage = (uint8_t)stage;
          r.sock = m.first;
          r.nmatch = (uint16_t)m.n;
          if (m.n > 1) flags |= OO_RX_F_MULTI;
        }
      }
    }
    r.reason = (uint8_t)reason;
    r.flags = flags;

    // ---- 5. stream the tile's long L4 regions as one flat chunk list.
    const uint32_t nc = longl4 ? (uint32_t)(((E4 + 15) >> 4) - HC) : 0u;
    const uint32_t incl = wave_scan(nc);
    const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    if (T != 0) {
      const uint32_t excl = incl - nc;
      // Chunk f of the flat list (f in [excl, incl) for this packet) is at
      // VB + 16 f with VB = abase + 16 (HC - excl); window position
      // 16 (f - excl + HC).
      const uint64_t vb = abase + (uint64_t)16 * ((uint64_t)HC - (uint64_t)excl);
      job[lane] = make_uint4((uint32_t)vb, (uint32_t)(vb >> 32), excl, (uint32_t)E4);

      // Buffers of SP pieces of 64 chunks (1 KiB each) into registers, two
      // buffers in flight: one buffer's loads land while the other is
      // reduced.  Every load is unconditional (lanes past the list reload
      // the last chunk, an L2 hit) so the compiler's vmcnt waits are static.
      //
      // Chunk -> packet: the packets whose run starts inside the buffer mark
      // their first chunk in kmap (job lane + 1); a max-scan over the marks,
      // carried across pieces and buffers (kc), gives every chunk's packet.
      //
      // Per-packet sums: G = running sum of the flat list (mod 2^32); the
      // chunk that starts a packet's run records G before it, the one that
      // ends it records G after it, so sum = g_end - g_start.  Plain LDS
      // writes, nothing to wait for inside the stream.
      uint32_t kc = 1;  // mark (job lane + 1) of the packet running into the next buffer
      uint32_t G = 0;   // running sum of the flat list before the buffer being reduced
      // meta per piece: job lane (7 bits) | chunk index in the run (10) | run end E4 (14);
      // all ones = past the list.
      auto issue = [&](uint4 (&buf)[SP], uint32_t F0, uint32_t (&meta)[SP]) {
        const uint32_t ln = opaque((uint32_t)lane);
        const uint32_t ex = opaque(excl);
#pragma unroll
        for (int w = 0; w < SP / 4; ++w) reinterpret_cast<uint32_t*>(kmap)[w * 64 + ln] = 0;
        if (nc != 0 && ex >= F0 && ex < F0 + SP * 64) kmap[ex - F0] = (uint8_t)(ln + 1);
        wave_sync_lds();
        uint32_t m[SP];
#pragma unroll
        for (int u = 0; u < SP; ++u) m[u] = kmap[u * 64 + ln];
#pragma unroll
        for (int u = 0; u < SP; ++u) {
          m[u] = max(wave_max_scan(m[u]), kc);
          kc = (uint32_t)__builtin_amdgcn_readlane((int)m[u], 63);
        }
        uint4 jk[SP];
#pragma unroll
        for (int u = 0; u < SP; ++u) jk[u] = job[m[u] - 1];
#pragma unroll
        for (int u = 0; u < SP; ++u) {
          const uint32_t f = F0 + ln + (uint32_t)(u * 64);
          const uint32_t fc = f < T ? f : T - 1;
          const uint64_t src = (((uint64_t)jk[u].y << 32) | jk[u].x) + (uint64_t)16 * fc;
          buf[u] = ld_stream(src);
          meta[u] = f < T ? (m[u] - 1) | ((f - jk[u].z) << 7) | (jk[u].w << 17) : 0xffffffffu;
        }
      };
      auto consume = [&](const uint4 (&buf)[SP], const uint32_t (&meta)[SP]) {
#pragma unroll
        for (int u = 0; u < SP; ++u) {
          const uint32_t mt = meta[u];
          const bool live = mt != 0xffffffffu;
          const uint32_t kf = mt & 127u;
          const int p = (int)(((mt >> 7) & 1023u) + HC) * 16;
          const int e4 = (int)(mt >> 17);
          uint32_t val = 0;
          if (live) val = p + 16 <= e4 ? chunk_sum_all(buf[u], 0u) : chunk_sum(buf[u], p, 0, e4);
          const uint32_t sc = wave_scan(val);
          const uint32_t g = G + sc;
          if (live && p == HC * 16) g_start[kf] = g - val;
          if (live && p + 16 >= e4) g_end[kf] = g;
          G += (uint32_t)__builtin_amdgcn_readlane((int)sc, 63);
        }
      };
      uint4 ba[SP], bb[SP];
      uint32_t ma[SP], mb[SP];
      constexpr uint32_t R = SP * 64;  // chunks per buffer
      issue(ba, 0, ma);
      issue(bb, R, mb);
      for (uint32_t F = 0; F < T; F += 2 * R) {
        // sched_barrier: keep each buffer's reloads after its reduction, so
        // only two buffers are ever live.
        consume(ba, ma);
        __builtin_amdgcn_sched_barrier(0);
        issue(ba, F + 2 * R, ma);
        __builtin_amdgcn_sched_barrier(0);
        consume(bb, mb);
        __builtin_amdgcn_sched_barrier(0);
        issue(bb, F + 3 * R, mb);
        __builtin_amdgcn_sched_barrier(0);
      }
      wave_sync_lds();
      const uint32_t jacc = longl4 ? g_end[lane] - g_start[lane] : 0u;
      s4 += jacc;
      if (longl4) {
        // The verdict the speculative record waited for; a failure turns it
        // into the drop record (only the fields a drop defines survive).
        uint32_t f = fold16(s4);
        if (shift & 1) f = swap16(f);
        if (fold16(f + pseudo) != 0xffffu) {
          r.reason = (uint8_t)(proto == 6u ? OO_RX_R_TCP_CSUM : OO_RX_R_UDP_CSUM);
          r.flags = (uint8_t)(flags & (OO_RX_F_VLAN | OO_RX_F_IP6));
          r.stage = 0; r.l4_off = 0; r.sport_be = 0; r.dport_be = 0; r.nmatch = 0;
          r.saddr_be = 0; r.daddr_be = 0; r.sock = -1; r.hash3 = 0;
        }
      }
    }


    if (valid) {
      uint4* o = reinterpret_cast<uint4*>(P.out + idx);
      const uint4* src = reinterpret_cast<const uint4*>(&r);
      o[0] = src[0];
      o[1] = src[1];
      atomicAdd(&ctr[r.reason & (OO_RX_R_COUNT - 1)], 1u);
    }
    wave_sync_lds();  // LDS is restaged by the next tile
  }

  __syncthreads();
  if (P.counters != nullptr && threadIdx.x < OO_RX_R_COUNT && ctr[threadIdx.x] != 0)
    atomicAdd(&P.counters[threadIdx.x], ctr[threadIdx.x]);
}

}  // namespace oo_rx

// Resident blocks per CU (sizes the persistent grid).
extern "C" int oo_rx_blocks_per_cu(void) {
  int b = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, oo_rx::rx_kernel, oo_rx::WAVES * 64, 0) !=
      hipSuccess)
    return 0;
  return b;
}

extern "C" int oo_rx_waves_per_block(void) { return oo_rx::WAVES; }

// Launch one batch on `stream`.
extern "C" int oo_rx_launch(const oo_rx::KParams* P, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(oo_rx::rx_kernel, dim3(grid), dim3(oo_rx::WAVES * 64), 0, stream, *P);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
