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
// Two kernels per batch (DESIGN.md "Kernels"):
//
// rx_head -- latency-bound per-packet work, one packet per lane, tiles of 64
//   packets per wave:
//   1. one coalesced 16-B descriptor load per lane (the next tile's is
//      prefetched while this one is processed);
//   2. the first 128 window bytes of the 64 frames are read with coalesced
//      16-B loads (8 lanes x 16 B per frame per instruction) and written
//      transposed into LDS as [chunk][packet] cells;
//   3. every lane parses its own packet from LDS (VLAN, IPv4/IPv6 gates, L4
//      gates, pseudo-header) and sums the IPv4 header and the part of the L4
//      region inside the window;
//   4. a packet whose L4 region ends inside the window gets its final
//      verdict here; one whose region runs past it is handled
//      speculatively as "checksum correct" and emits a 16-byte tail job;
//   5. IPv4 frag/options/TCP-scattered tests, the 2 or 3 filter-table
//      lookup stages (first probes of all stages issued together), and the
//      32-byte record.
//
// rx_tail -- bandwidth-bound streaming of the long L4 regions, 16 lanes (one
//   DPP row) per job, 8 x 16-B nontemporal loads per lane in flight, sums by
//   v_dot2_u32_u16 and a DPP row reduction; a failed checksum rewrites the
//   speculative record (a drop keeps only the fields a drop defines) and
//   moves one count between the per-reason counters.
//
// The verdict uses the mod-0xffff residue of the exact word sum; see
// oracle/rx_oracle.c for why that equals the reference's folded-complement
// test, and why the sum splits into head + tail parts.  No MFMA: integer
// reduction + table probes, HBM-bound.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "oo_rx_device.h"

namespace oo_rx {

typedef unsigned short v2u16 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int HEAD_WAVES = HEAD_WAVES_PER_BLOCK;  // waves per rx_head block
constexpr int TAIL_WAVES = 4;        // waves per rx_tail block
constexpr int HC = 8;                // staged header chunks per packet
constexpr int HB = HC * 16;          // staged window bytes per packet
constexpr int ROWB = 64 * 16 + 16;   // one staged chunk of all 64 packets (+pad)
constexpr int SG = 16;               // lanes per tail job (one DPP row)
constexpr int SU = 8;                // 16-B chunks per lane per tail round

// Filter-table entry states (netif_table.c:34-42).
constexpr uint32_t ST_MASK = 0xc0000000u;
constexpr uint32_t ID_MASK = 0x3fffffffu;
constexpr uint32_t ST_PREFERRED = 0x00000000u;
constexpr uint32_t ST_EMPTY = 0x80000000u;
constexpr uint32_t ST_TOMBSTONE = 0xc0000000u;
constexpr int ID6_EMPTY = -2;
constexpr uint32_t PENDING = 0xffu;

__device__ __forceinline__ uint4 ld_stream(const uint4* p) {
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
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

// ---------------------------------------------------------------------------
// rx_head

struct HeadLds {
  uint8_t hdr[HC][ROWB];  // staged headers, [chunk][packet] 16-B cells
};

__global__ __launch_bounds__(HEAD_WAVES * 64) void rx_head(KParams P) {
  __shared__ __attribute__((aligned(16))) HeadLds lds[HEAD_WAVES];
  __shared__ uint32_t ctr[OO_RX_R_COUNT];

  const int wave = (int)(threadIdx.x >> 6);
  const int lane = (int)(threadIdx.x & 63);
  HeadLds& L = lds[wave];
  if (threadIdx.x < OO_RX_R_COUNT) ctr[threadIdx.x] = 0;
  __syncthreads();

  const uint32_t ntiles = (P.n + 63) / 64;
  const uint32_t stride = gridDim.x * HEAD_WAVES;
  uint32_t tile = blockIdx.x * HEAD_WAVES + wave;
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
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int f = kk * 8 + (lane >> 3);
      const int c = lane & 7;
      const uint32_t ablo = (uint32_t)__shfl((int)(uint32_t)abase, f, 64);
      const uint32_t abhi = (uint32_t)__shfl((int)(uint32_t)(abase >> 32), f, 64);
      const int sp = __shfl(span, f, 64);
      if (c * 16 < sp) {
        const uint4* src = reinterpret_cast<const uint4*>(((uint64_t)abhi << 32) | ablo) + c;
        *reinterpret_cast<uint4*>(&L.hdr[c][f * 16]) = ld_stream(src);
      }
    }
    wave_sync_lds();

    const uint8_t* my = &L.hdr[0][lane * 16];
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
    wave_sync_lds();  // the staging cells are refilled by the next tile

    // ---- 4. verdict (or a tail job).
    if (reason == PENDING && need_ip) {
      // IHL != 0 makes the word sum non-zero: fold == 0xffff <=> valid.
      if (ihl4 == 0 || fold16(s3) != 0xffffu) reason = OO_RX_R_IP4_CSUM;
    }
    if (reason == PENDING && l4_gate != PENDING) reason = l4_gate;
    bool job = false;
    uint32_t cres = 0;
    if (reason == PENDING && need_l4) {
      uint32_t f = fold16(s4);
      if (shift & 1) f = swap16(f);  // RFC 1071 byte-order swap
      cres = fold16(f + pseudo);
      if (E4 > HB) job = true;  // verdict pending on the tail
      else if (cres != 0xffffu) reason = proto == 6u ? OO_RX_R_TCP_CSUM : OO_RX_R_UDP_CSUM;
    }
    {
      const uint64_t mj = __ballot(job);
      if (mj != 0) {
        // One append per wave to this wave's job shard (64 shards, no hot
        // counter: a single device-wide counter saturates near 88 adds/us).
        const uint32_t shard = (blockIdx.x * HEAD_WAVES + (uint32_t)wave) % JOB_SHARDS;
        uint32_t jbase = 0;
        if (lane == 0) jbase = atomicAdd(&P.njobs[shard * JOB_CTR_STRIDE], (uint32_t)__popcll(mj));
        jbase = (uint32_t)__shfl((int)jbase, 0, 64);
        if (job) {
          const uint32_t below = __builtin_amdgcn_mbcnt_hi(
              (uint32_t)(mj >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mj, 0));
          uint4* J = reinterpret_cast<uint4*>(P.jobs) + (uint64_t)shard * P.job_cap + jbase + below;
          *J = make_uint4((uint32_t)abase, (uint32_t)(abase >> 32),
                          idx | ((uint32_t)(shift & 1) << 31),
                          (cres << 16) | (uint32_t)(E4 - HB));
        }
      }
    }

    // ---- 5. handle_rx_pkt, demux, record (per lane).
    oo_gpu_rx_result r;
    r.reason = 0; r.flags = 0; r.stage = 0; r.proto = 0; r.vlan = (uint16_t)vlan;
    r.l4_off = 0; r.ip_paylen = 0; r.sport_be = 0; r.dport_be = 0; r.nmatch = 0;
    r.saddr_be = 0; r.daddr_be = 0; r.sock = -1; r.hash3 = 0;
    if (l3ok) {
      r.proto = (uint8_t)proto;
      r.ip_paylen = (uint16_t)ip_paylen;
    }

    if (reason == PENDING) {
      // handled: handle_rx_pkt (netif_event.c:250-451)
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
          const Ip6Entry e0 = P.ip6[h1_0];
          const Ip6Entry e1 = P.ip6[h1_1];
          Ip6Entry e2 = e1;
          if (nst == 3) e2 = P.ip6[h1_2];
          m = walk6(P, a6d, dport, a6s, false, sport, proto, intf_i, vlan, h1_0, e0);
          stage = 1;
          if (m.n == 0) {
            m = walk6(P, a6d, dport, zero, true, 0u, proto, intf_i, vlan, h1_1, e1);
            stage = 2;
          }
          if (m.n == 0 && nst == 3) {
            m = walk6(P, zero, dport, zero, true, 0u, proto, intf_i, vlan, h1_2, e2);
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

    if (valid) {
      uint4* o = reinterpret_cast<uint4*>(P.out + idx);
      const uint4* src = reinterpret_cast<const uint4*>(&r);
      o[0] = src[0];
      o[1] = src[1];
      atomicAdd(&ctr[reason & (OO_RX_R_COUNT - 1)], 1u);
    }
  }

  __syncthreads();
  if (P.counters != nullptr && threadIdx.x < OO_RX_R_COUNT && ctr[threadIdx.x] != 0)
    atomicAdd(&P.counters[threadIdx.x], ctr[threadIdx.x]);
}

// ---------------------------------------------------------------------------
// rx_tail

__global__ __launch_bounds__(TAIL_WAVES * 64) void rx_tail(KParams P) {
  // Prefix over the job shards' counts: job v lives in shard s with
  // pref[s] <= v < pref[s+1], at entry v - pref[s] of that shard.
  __shared__ uint32_t pref[JOB_SHARDS + 1];
  __shared__ __attribute__((aligned(16))) uint4 ring[TAIL_WAVES][SU][64];
  if (threadIdx.x < JOB_SHARDS) {
    const uint32_t c = __hip_atomic_load(&P.njobs[threadIdx.x * JOB_CTR_STRIDE], __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    uint32_t x = c;
#pragma unroll
    for (int o = 1; o < JOB_SHARDS; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
      if ((int)threadIdx.x >= o) x += y;
    }
    pref[threadIdx.x + 1] = x;
    if (threadIdx.x == 0) pref[0] = 0;
  }
  __syncthreads();
  const uint32_t njobs = pref[JOB_SHARDS];
  const int wave = (int)(threadIdx.x >> 6);
  const int lane = (int)(threadIdx.x & 63);
  const int gl = lane & (SG - 1);
  const uint32_t group = (blockIdx.x * TAIL_WAVES + (uint32_t)wave) * (64 / SG) +
                         (uint32_t)(lane / SG);
  const uint32_t stride = gridDim.x * TAIL_WAVES * (64 / SG);
  const uint4* jobs = reinterpret_cast<const uint4*>(P.jobs);

  auto load_job = [&](uint32_t v) -> uint4 {
    uint32_t sh = 0;
#pragma unroll
    for (uint32_t step = JOB_SHARDS / 2; step; step >>= 1)
      if (pref[sh + step] <= v) sh += step;
    return jobs[(uint64_t)sh * P.job_cap + (v - pref[sh])];
  };
  uint4 jnext = group < njobs ? load_job(group) : make_uint4(0, 0, 0, 0);
  for (uint32_t j = group; j < njobs; j += stride) {
    // This round's job descriptor was loaded during the previous round;
    // fetch the next one now so no round starts on a dependent load.
    const uint4 jb = jnext;
    if (j + stride < njobs) jnext = load_job(j + stride);
    const uint4* ab = reinterpret_cast<const uint4*>(((uint64_t)jb.y << 32) | jb.x);
    const int e4 = (int)(jb.w & 0xffffu) + HB;  // window end of the L4 region
    const int nch = (e4 + 15) >> 4;
    uint32_t acc = 0;
    for (int c0 = HC; c0 < nch; c0 += SG * SU) {
      // LDS-DMA (global_load_lds_dwordx4, nontemporal): lane l's 16 bytes
      // land in cell l of ring slot u; the lane reads its own cell back.
      // Cells of chunks past the region are never loaded and sum to 0.
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int c = c0 + gl + SG * u;
        if (c < nch)
          __builtin_amdgcn_global_load_lds(
              (const void*)(ab + c), (void __attribute__((address_space(3)))*)&ring[wave][u][0], 16,
              0, 2 /* nt */);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int c = c0 + gl + SG * u;
        const uint4 v = ring[wave][u][lane];
        if (c * 16 + 16 <= e4) acc = chunk_sum_all(v, acc);
        else acc += chunk_sum(v, c * 16, 0, e4);
      }
      __builtin_amdgcn_wave_barrier();  // the ring is refilled next round
    }
    acc = row_sum16(acc);
    if (gl == SG - 1) {
      uint32_t f = fold16(acc);
      if (jb.z >> 31) f = swap16(f);
      if (fold16(f + (jb.w >> 16)) != 0xffffu) {
        // Checksum failed: the speculative record becomes a drop, which keeps
        // only vlan, the VLAN/IP6 flags, proto and ip_paylen.
        const uint32_t idx = jb.z & 0x7fffffffu;
        uint4* o = reinterpret_cast<uint4*>(P.out + idx);
        const uint4 w0 = o[0];
        const uint32_t old_reason = w0.x & 0xffu;
        const uint32_t proto = (w0.x >> 24) & 0xffu;
        const uint32_t nr = proto == 6u ? OO_RX_R_TCP_CSUM : OO_RX_R_UDP_CSUM;
        const uint32_t fl = (w0.x >> 8) & (OO_RX_F_VLAN | OO_RX_F_IP6);
        o[0] = make_uint4(nr | (fl << 8) | (proto << 24), w0.y & 0xffffu,  // vlan
                          w0.z & 0xffffu,                                    // ip_paylen
                          0);
        o[1] = make_uint4(0, 0, 0xffffffffu, 0);                             // sock = -1
        if (P.counters != nullptr) {
          atomicSub(&P.counters[old_reason & (OO_RX_R_COUNT - 1)], 1u);
          atomicAdd(&P.counters[nr], 1u);
        }
      }
    }
  }
}

}  // namespace oo_rx

// Resident blocks per CU of each kernel (sizes the persistent grids).
extern "C" int oo_rx_shape(int n_cu, oo_rx::LaunchShape* s) {
  int h = 0, t = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&h, oo_rx::rx_head, oo_rx::HEAD_WAVES * 64,
                                                   0) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&t, oo_rx::rx_tail, oo_rx::TAIL_WAVES * 64,
                                                   0) != hipSuccess)
    return -1;
  s->head_grid = n_cu * (h > 0 ? h : 1);
  s->tail_grid = n_cu * (t > 0 ? t : 1);
  return 0;
}

// Launch wrappers used by the C-ABI layer (oo_gpu_rx.cpp): the head, then
// (after the head, on the same or an event-chained stream) the tail.  The
// job-shard counters must be zeroed before the head.
extern "C" int oo_rx_launch_head(const oo_rx::KParams* P, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(oo_rx::rx_head, dim3(grid), dim3(oo_rx::HEAD_WAVES * 64), 0, stream, *P);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
extern "C" int oo_rx_launch_tail(const oo_rx::KParams* P, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(oo_rx::rx_tail, dim3(grid), dim3(oo_rx::TAIL_WAVES * 64), 0, stream, *P);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int oo_rx_tail_groups_per_block(void) { return oo_rx::TAIL_WAVES * (64 / oo_rx::SG); }
