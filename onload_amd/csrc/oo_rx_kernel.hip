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
// Execution model (DESIGN.md "Kernel"): each wave owns tiles of 64 packets,
// one packet per lane for everything that is per-packet and latency-bound,
// and 16-lane rows for the byte stream:
//
//  1. one coalesced 16-B descriptor load per lane;
//  2. header staging: the first 128 window bytes of the 64 frames are read
//     with coalesced 16-B loads (8 lanes x 16 B per frame per instruction)
//     and written transposed into LDS as [chunk][packet] cells, so that
//  3. every lane parses its own packet's headers from LDS (VLAN, IPv4/IPv6
//     gates, L4 gates, pseudo-header) and sums the IPv4 header and the part
//     of the L4 region inside those 128 bytes;
//  4. packets whose L4 region extends past 128 bytes are streamed by 16-lane
//     rows (4 packets at a time per wave), 8 x 16-B loads per lane in flight,
//     one's-complement partial sums by v_dot2_u32_u16 and a DPP row
//     reduction (no LDS traffic);
//  5. every lane finishes its packet: verdict, IPv4 frag/options/TCP
//     scattered tests, the 2 or 3 filter-table lookup stages
//     (double-hashed probe walks, all 64 lanes' walks in flight together),
//     and one 32-byte record.
//  Per-reason counters accumulate in LDS and are flushed once per block.
//
// The one's-complement verdict uses the mod-0xffff residue of the exact word
// sum; oracle/rx_oracle.c explains why it equals the reference's
// folded-complement test.  No MFMA: integer reduction + table probes,
// HBM-bound.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "oo_rx_device.h"

namespace oo_rx {

typedef unsigned short v2u16 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int WAVES = 4;             // waves per block
constexpr int HC = 8;                // staged header chunks per packet
constexpr int HB = HC * 16;          // staged window bytes per packet
constexpr int ROWB = 64 * 16 + 16;   // one staged chunk of all 64 packets (+pad)
constexpr int SG = 16;               // lanes per streaming group (one DPP row)
constexpr int SU = 8;                // 16-B chunks per lane per streaming round

// Filter-table entry states (netif_table.c:34-42).
constexpr uint32_t ST_MASK = 0xc0000000u;
constexpr uint32_t ID_MASK = 0x3fffffffu;
constexpr uint32_t ST_PREFERRED = 0x00000000u;
constexpr uint32_t ST_EMPTY = 0x80000000u;
constexpr uint32_t ST_TOMBSTONE = 0xc0000000u;
constexpr int ID6_EMPTY = -2;
constexpr uint32_t PENDING = 0xffu;

struct WaveLds {
  uint8_t hdr[HC][ROWB];  // staged headers, [chunk][packet] 16-B cells
  uint4 meta[64];         // streaming job: {abase lo, abase hi, E4, -}
  uint32_t ssum[64];      // streamed L4 partial sums
  uint8_t jobs[64];       // streaming job list (lane ids)
};

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

// ci_netif_filter_for_each_match (netif_table.c:234-319).
__device__ Match walk4(const KParams& P, uint32_t la, uint32_t lp, uint32_t ra, uint32_t rp,
                       uint32_t proto, int intf_i, int vlan) {
  Match m = {-1, 0};
  const uint32_t mask = P.ip4_mask;
  uint32_t h1 = hash3(la, lp, ra, rp, proto) & mask;
  const uint32_t first = h1;
  const uint32_t h2 = hash2(la, lp, ra, rp, proto);
  uint2 e = P.ip4[h1];
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

// ci_netif_filter_for_each_match_ip6 (netif_table_ip6.c:110-189).
__device__ Match walk6(const KParams& P, const uint32_t la[4], uint32_t lp, const uint32_t ra[4],
                       bool ra_null, uint32_t rp, uint32_t proto, int intf_i, int vlan) {
  Match m = {-1, 0};
  const uint32_t mask = P.ip6_mask;
  const uint32_t lx = la[0] ^ la[1] ^ la[2] ^ la[3];
  const uint32_t rx = ra_null ? 0u : (ra[0] ^ ra[1] ^ ra[2] ^ ra[3]);
  uint32_t h1 = hash3(lx, lp, rx, rp, proto) & mask;
  const uint32_t first = h1;
  const uint32_t h2 = hash2(lx, lp, rx, rp, proto);
  for (uint32_t guard = 0; guard <= mask; ++guard) {
    const Ip6Entry e = P.ip6[h1];
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
  }
  return m;
}

// ---------------------------------------------------------------------------

__global__ __launch_bounds__(WAVES * 64) void rx_kernel(KParams P) {
  __shared__ __attribute__((aligned(16))) WaveLds lds[WAVES];
  __shared__ uint32_t ctr[OO_RX_R_COUNT];

  const int wave = (int)(threadIdx.x >> 6);
  const int lane = (int)(threadIdx.x & 63);
  WaveLds& L = lds[wave];
  if (threadIdx.x < OO_RX_R_COUNT) ctr[threadIdx.x] = 0;
  __syncthreads();

  const uint32_t ntiles = (P.n + 63) / 64;
  const uint32_t stride = gridDim.x * WAVES;
  for (uint32_t tile = blockIdx.x * WAVES + wave; tile < ntiles; tile += stride) {
    // ---- 1. descriptor (one per lane)
    const uint32_t idx = tile * 64 + (uint32_t)lane;
    const bool valid = idx < P.n;
    uint4 d = make_uint4(0, 0, 0, 0);
    if (valid) d = ld_stream(reinterpret_cast<const uint4*>(P.desc) + idx);
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
    auto B = [&](int j) -> uint32_t {
      if (j < 0 || j >= len) return 0u;
      const int w = shift + j;
      return (uint32_t)my[(w >> 4) * ROWB + (w & 15)];
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

    // ---- 4. stream the rest of long L4 regions with 16-lane rows.
    const bool job = need_l4 && E4 > HB;
    const uint64_t mj = __ballot(job);
    if (mj != 0) {
      const uint32_t below = __builtin_amdgcn_mbcnt_hi(
          (uint32_t)(mj >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mj, 0));
      if (job) {
        L.jobs[below] = (uint8_t)lane;
        L.meta[lane] = make_uint4((uint32_t)abase, (uint32_t)(abase >> 32), (uint32_t)E4, 0);
      }
      wave_sync_lds();
      const int nj = __popcll(mj);
      const int g = lane >> 4, gl = lane & 15;
      for (int j = g; j < nj; j += 64 / SG) {
        const int jl = L.jobs[j];
        const uint4 mt = L.meta[jl];
        const uint4* ab = reinterpret_cast<const uint4*>(((uint64_t)mt.y << 32) | mt.x);
        const int e4 = (int)mt.z;
        const int nch = (e4 + 15) >> 4;
        uint32_t acc = 0;
        for (int c0 = HC; c0 < nch; c0 += SG * SU) {
          uint4 v[SU];
#pragma unroll
          for (int u = 0; u < SU; ++u) {
            const int c = c0 + gl + SG * u;
            v[u] = c < nch ? ld_stream(ab + c) : make_uint4(0, 0, 0, 0);
          }
#pragma unroll
          for (int u = 0; u < SU; ++u) {
            const int c = c0 + gl + SG * u;
            if (c * 16 + 16 <= e4) acc = chunk_sum_all(v[u], acc);
            else acc += chunk_sum(v[u], c * 16, 0, e4);
          }
        }
        acc = row_sum16(acc);
        if (gl == 15) L.ssum[jl] = acc;
      }
      wave_sync_lds();
      if (job) s4 += L.ssum[lane];
    }

    // ---- 5. verdict, handle_rx_pkt, demux, record (per lane).
    if (reason == PENDING && need_ip) {
      // IHL != 0 makes the word sum non-zero: fold == 0xffff <=> valid.
      if (ihl4 == 0 || fold16(s3) != 0xffffu) reason = OO_RX_R_IP4_CSUM;
    }
    if (reason == PENDING && l4_gate != PENDING) reason = l4_gate;
    if (reason == PENDING && need_l4) {
      uint32_t f = fold16(s4);
      if (shift & 1) f = ((f & 0xffu) << 8) | (f >> 8);  // RFC 1071 byte-order swap
      if (fold16(f + pseudo) != 0xffffu)
        reason = proto == 6u ? OO_RX_R_TCP_CSUM : OO_RX_R_UDP_CSUM;
    }

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
        // Demux stages in reference order (udp_rx.c:271-306, tcp_rx.c:4786-4835);
        // the first stage with a match decides.
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
        for (int s = 0; s < nst && m.n == 0; ++s) {
          if (is6) {
            const uint32_t zero[4] = {0, 0, 0, 0};
            m = walk6(P, s == 2 ? zero : a6d, dport, s == 0 ? a6s : zero, s != 0,
                      s == 0 ? sport : 0u, proto, intf_i, vlan);
          } else {
            m = walk4(P, s == 2 ? 0u : r.daddr_be, dport, s == 0 ? r.saddr_be : 0u,
                      s == 0 ? sport : 0u, proto, intf_i, vlan);
          }
          stage = s + 1;
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
    wave_sync_lds();  // staging buffers are reused by the next tile
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

// Launch wrapper used by the C-ABI layer.
extern "C" int oo_rx_launch(const oo_rx::KParams* P, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(oo_rx::rx_kernel, dim3(grid), dim3(oo_rx::WAVES * 64), 0, stream, *P);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
