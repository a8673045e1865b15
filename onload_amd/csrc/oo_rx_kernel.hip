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
// One persistent kernel, rx_kernel (DESIGN.md "Kernel").  Each wave owns
// tiles of 64 packets (one packet per lane for parse/demux) and strides over
// them.  Every HBM read of frame bytes and descriptors is an LDS-DMA
// (global_load_lds_dwordx4, nontemporal) whose completion the wave counts
// itself with `s_waitcnt vmcnt(N)`; only the filter-table probes are plain
// loads.  Per tile:
//   1. descriptors: one 1-KiB LDS-DMA piece (the next tile's is issued as
//      soon as this one is read);
//   2. header window: the first 128 bytes of each frame, 8 pieces, lane =
//      packet, landing transposed as [chunk][packet] 16-B cells;
//   3. body: the frame bytes past the window, streamed through a ring of R
//      1-KiB slots.  Eight lanes (an 8-lane group, 128 contiguous bytes per
//      round) stream one packet at a time; the tile's packets with a body are
//      dealt round-robin to the wave's eight groups.  The first R pieces are
//      issued before the parse, so they land while it runs;
//   4. per lane: VLAN, L3/L4 gates, pseudo-header, window sums, handle_rx_pkt's
//      frag/options/TCP-scattered tests, the 2 or 3 lookup stages, a
//      speculative 32-B record;
//   5. the body stream: every lane sums its 16-B chunk (masked at the L4
//      region end), accumulates per packet, and an 8-lane DPP reduction hands
//      each packet's body sum to its parse lane, which then decides the
//      verdict the record waited for.
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
#ifndef OO_RX_RING
#define OO_RX_RING 6
#endif
#ifndef OO_RX_WPE
#define OO_RX_WPE 0  // amdgpu_waves_per_eu target, 0 = compiler's choice
#endif

constexpr int WAVES = OO_RX_WAVES;   // waves per block
constexpr int R = OO_RX_RING;        // body ring slots (1 KiB each) per wave
constexpr int HC = 8;                // staged header chunks per packet
constexpr int HB = HC * 16;          // staged window bytes per packet
constexpr int ROWB = 64 * 16;        // one staged chunk of all 64 packets
constexpr uint32_t M_LIVE = 1u << 16;  // body meta: chunk inside the frame
constexpr uint32_t M_LAST = 1u << 17;  // body meta: the group's last round of the packet

// Filter-table entry states (netif_table.c:34-42).
constexpr uint32_t ST_MASK = 0xc0000000u;
constexpr uint32_t ID_MASK = 0x3fffffffu;
constexpr uint32_t ST_PREFERRED = 0x00000000u;
constexpr uint32_t ST_EMPTY = 0x80000000u;
constexpr uint32_t ST_TOMBSTONE = 0xc0000000u;
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

// Value of v in lane src (ds_bpermute: no LDS memory access, so it needs no
// vmcnt wait).  Call with every lane active.
__device__ __forceinline__ uint32_t lane_get(uint32_t v, uint32_t src) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v);
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

#ifdef OO_RX_STAMPS
// Diagnostic phase stamps: stamps[((wave * 64 + iter) * 8) + phase] = realtime
// (100 MHz) for the first 64 tiles of each wave.
#define STAMP(ph, val)                                                                \
  do {                                                                                \
    if (P.stamps != nullptr && lane == 0 && it_ < 64)                                \
      P.stamps[((size_t)gwave * 64 + it_) * 8 + (ph)] = (val);                        \
  } while (0)
#else
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

// ---------------------------------------------------------------------------
// Demux: one lookup stage walked to its end (every match counted).

struct Match {
  int32_t first;
  uint32_t n;
};

__device__ __forceinline__ bool occ_bit(const uint32_t* occ, uint32_t i) {
  return ((occ[i >> 5] >> (i & 31u)) & 1u) != 0;
}

// ci_sock_intf_check (netif_table.h:30-36) on the socket fields of a slot.
__device__ __forceinline__ bool bind2dev_ok(const KParams& P, uint32_t sflags, uint64_t hwports,
                                            int b2d_vlan, int intf_i, int vlan) {
  if (!(sflags & OO_GPU_RX_SOCK_BIND2DEV)) return true;
  const uint32_t hw =
      (intf_i >= 0 && intf_i < OO_GPU_RX_MAX_INTF) ? P.hwport[intf_i] : 0xffu;
  return hw < 64 && (hwports & (1ull << hw)) != 0 && b2d_vlan == vlan;
}

__device__ __forceinline__ Slot4 load_slot4(const KParams& P, uint32_t i) {
  const uint4* p = reinterpret_cast<const uint4*>(P.slot4 + i);
  Slot4 r;
  uint4* d = reinterpret_cast<uint4*>(&r);
  d[0] = p[0];
  d[1] = p[1];
  return r;
}
__device__ __forceinline__ Slot6 load_slot6(const KParams& P, uint32_t i) {
  const uint4* p = reinterpret_cast<const uint4*>(P.slot6 + i);
  Slot6 r;
  uint4* d = reinterpret_cast<uint4*>(&r);
  d[0] = p[0];
  d[1] = p[1];
  d[2] = p[2];
  d[3] = p[3];
  return r;
}

// ci_netif_filter_for_each_match (netif_table.c:234-319) over the slot
// records, every match counted.  The caller has loaded the not-EMPTY bits of
// the first slot (occ) and of the next one on the probe sequence (occ_next),
// and the first slot's record when occ: the common walk (an EMPTY first
// slot, or one occupied slot followed by an EMPTY one) needs no more loads.
__device__ Match walk4(const KParams& P, uint32_t la, uint32_t lp, uint32_t ra, uint32_t rp,
                       uint32_t proto, int intf_i, int vlan, uint32_t h1, uint32_t h2, bool occ,
                       Slot4 rec, bool occ_next) {
  Match m = {-1, 0};
  const uint32_t mask = P.ip4_mask;
  const uint32_t first = h1;
  bool check_lport = false;  // the first slot's lport is implied (LPRP, hash.h:76-163)
  for (uint32_t guard = 0; guard <= mask; ++guard) {
    if (!occ) break;  // an EMPTY slot ends the walk
    const uint32_t st = rec.id_state & ST_MASK;
    if ((check_lport ? occupied(st) : st == ST_PREFERRED) && rec.laddr == la &&
        rec.raddr == ra && rec.rport == rp && rec.proto == proto &&
        (!check_lport || rec.lport == lp) &&
        bind2dev_ok(P, rec.sflags, rec.hwports, rec.b2d_vlan, intf_i, vlan)) {
      if (m.n == 0) m.first = (int32_t)(rec.id_state & ID_MASK);
      ++m.n;
    }
    h1 = (h1 + h2) & mask;
    if (h1 == first) break;
    occ = guard == 0 ? occ_next : occ_bit(P.occ4, h1);
    if (occ) rec = load_slot4(P, h1);
    check_lport = true;
  }
  return m;
}

// ci_netif_filter_for_each_match_ip6 (netif_table_ip6.c:110-189) over the
// slot records; same first-slot convention as walk4.
__device__ Match walk6(const KParams& P, const uint32_t la[4], uint32_t lp, const uint32_t ra[4],
                       bool ra_null, uint32_t rp, uint32_t proto, int intf_i, int vlan,
                       uint32_t h1, uint32_t h2, bool occ, Slot6 rec, bool occ_next) {
  Match m = {-1, 0};
  const uint32_t mask = P.ip6_mask;
  const uint32_t first = h1;
  for (uint32_t guard = 0; guard <= mask; ++guard) {
    if (!occ) break;  // an EMPTY slot ends the walk (tombstones continue)
    if (rec.id >= 0 && rec.laddr[0] == la[0] && rec.laddr[1] == la[1] &&
        rec.laddr[2] == la[2] && rec.laddr[3] == la[3] && rec.lport == lp &&
        rec.proto == proto &&
        (ra_null ? !(rec.sflags & OO_GPU_RX_SOCK_CONNECTED)
                 : (rec.raddr[0] == ra[0] && rec.raddr[1] == ra[1] && rec.raddr[2] == ra[2] &&
                    rec.raddr[3] == ra[3] && rec.rport == rp)) &&
        bind2dev_ok(P, rec.sflags, rec.hwports, rec.b2d_vlan, intf_i, vlan)) {
      if (m.n == 0) m.first = rec.id;
      ++m.n;
    }
    h1 = (h1 + h2) & mask;
    if (h1 == first) break;
    occ = guard == 0 ? occ_next : occ_bit(P.occ6, h1);
    if (occ) rec = load_slot6(P, h1);
  }
  return m;
}


// ---------------------------------------------------------------------------

#if OO_RX_WPE > 0
#define OO_RX_KATTR __attribute__((amdgpu_waves_per_eu(OO_RX_WPE)))
#else
#define OO_RX_KATTR
#endif

// Per-wave LDS.  All LDS lives in one __shared__ array (a second __shared__
// object can make hipcc wait vmcnt(0) before LDS reads while LDS-DMA is in
// flight).
struct WaveLds {
  uint4 hdr[HC][64];   // header window, [chunk][packet] 16-B cells
  uint4 ring[R][64];   // body ring: slot = one round of the eight groups
  uint4 desc[64];      // the tile's descriptors
};
static_assert(sizeof(WaveLds) % 16 == 0, "WaveLds is carved from a uint4 array");
constexpr int WAVE_U4 = (int)(sizeof(WaveLds) / 16);

__global__ __launch_bounds__(WAVES * 64) OO_RX_KATTR void rx_kernel(KParams P) {
  __shared__ __attribute__((aligned(16))) uint4 smem[WAVES * WAVE_U4 + OO_RX_R_COUNT / 4];

  const int wave = (int)(threadIdx.x >> 6);
  const int lane = (int)(threadIdx.x & 63);
  const uint32_t grp = (uint32_t)lane >> 3;  // 8-lane group
  const uint32_t gj = (uint32_t)lane & 7u;   // lane within the group
  WaveLds& L = reinterpret_cast<WaveLds*>(smem)[wave];
  uint32_t* ctr = reinterpret_cast<uint32_t*>(smem + WAVES * WAVE_U4);
  if (threadIdx.x < OO_RX_R_COUNT) ctr[threadIdx.x] = 0;
  __syncthreads();

  // Tiles of P.tile packets (<= 64), sized by the host so that every wave
  // gets the same number of tiles (oo_gpu_rx.cpp launch()).
  const uint32_t TS = P.tile;
  const uint32_t ntiles = (P.n + TS - 1) / TS;
  const uint32_t stride = gridDim.x * WAVES;
  uint32_t tile = blockIdx.x * WAVES + wave;
  // Lanes with nothing to load read this always-mapped 16-B line instead, so
  // every LDS-DMA instruction is issued by the whole wave and the counted
  // waits stay static.
  const uint64_t dummy = reinterpret_cast<uint64_t>(P.desc);
  const uint64_t descs = reinterpret_cast<uint64_t>(P.desc);
  auto issue_desc = [&](uint32_t t) {
    const uint32_t i = t * TS + (uint32_t)lane;
    glds((uint32_t)lane < TS && i < P.n ? descs + (uint64_t)i * 16 : dummy, &L.desc[0]);
  };
  if (tile < ntiles) issue_desc(tile);
  vm_wait<0>();
  const uint32_t gwave = blockIdx.x * WAVES + wave;
  uint32_t it_ = 0;
  (void)gwave;
  (void)it_;

  for (; tile < ntiles; tile += stride, ++it_) {
    STAMP(0, __builtin_amdgcn_s_memrealtime());
    STAMP(6, tile);
    // ---- 1. descriptor (landed: every earlier wait retired it), then the
    // next tile's.
    const uint32_t idx = tile * TS + (uint32_t)lane;
    const bool valid = (uint32_t)lane < TS && idx < P.n;
    const uint4 d = lds_read16(&L.desc[lane]);
    if (tile + stride < ntiles) issue_desc(tile + stride);
    const uint64_t off = (uint64_t)d.x | ((uint64_t)d.y << 32);
    int len = (int)(d.z & 0xffffu);
    const int intf_i = (int)(int16_t)(d.z >> 16);
    const bool inb = valid && off + (uint64_t)len <= P.frames_bytes;
    if (!inb) len = 0;  // a descriptor outside the buffer is an empty frame
    const uint64_t base = reinterpret_cast<uint64_t>(P.frames) + (inb ? off : 0);
    const int shift = (int)(base & 15u);
    const uint64_t abase = base - (uint64_t)shift;
    const int span = inb ? shift + len : 0;
    const int nwin = (span + 15) >> 4;  // 16-B chunks the frame touches

    // ---- 2. header window: chunk k of every frame, lane = packet.
#pragma unroll
    for (int k = 0; k < HC; ++k) glds<OO_RX_HDR_AUX>(k < nwin ? abase + (uint64_t)k * 16 : dummy, &L.hdr[k][0]);

    // ---- 3. body jobs.  The packets with chunks past the window, in lane
    // order, are list positions q = 0..M-1; group g takes q = g, g+8, ...
    // Lane (g, j) holds the job at q = g + 8 j (a permutation, so every lane
    // sends and receives exactly one value).
    const uint32_t nb = nwin > HC ? (uint32_t)(nwin - HC) : 0u;
    const uint64_t bm = __ballot(nb != 0);
    const uint32_t M = (uint32_t)__popcll(bm);
    const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32),
                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
    const uint32_t myq = nb != 0 ? below : M + (uint32_t)lane - below;
    const uint32_t myslot = (myq & 7u) * 8u + (myq >> 3);  // lane holding job myq
    const uint32_t jp = (uint32_t)__builtin_amdgcn_ds_permute((int)(myslot << 2), lane);
    const uint64_t bbase = abase + HB;
    const uint32_t jlo = lane_get((uint32_t)bbase, jp);
    const uint32_t jhi = lane_get((uint32_t)(bbase >> 32), jp);
    const uint32_t jnb = lane_get(nb, jp);  // 0 for lanes past the list
    // Rounds of the body stream = the busiest group's.
    const uint32_t gr = group_sum8((jnb + 7u) >> 3);
    uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)gr, 0);
#pragma unroll
    for (int g = 1; g < 8; ++g) T = max(T, (uint32_t)__builtin_amdgcn_readlane((int)gr, 8 * g));

    // Issue state: the group's job number ik, its packet ip, this lane's
    // chunk ic (= 8 * round + gj) out of inb_, and the source address.
    const uint32_t gsrc = grp * 8u;
    uint32_t ik = 0;
    uint32_t ip = lane_get(jp, gsrc), inb_ = lane_get(jnb, gsrc), ic = gj;
    uint64_t iaddr = ((uint64_t)lane_get(jhi, gsrc) << 32 | lane_get(jlo, gsrc)) + gj * 16u;
    // Per piece (slot u) and lane, meta[u] says what landed: before the
    // parse, {packet, chunk, live, last}; after it, {valid bytes nv (0..16)
    // of the chunk inside the packet's summed region, last}.
    uint32_t meta[R];
    uint32_t ilim = 0;  // summed-region end of the job being issued (after the parse)
    uint32_t lim_mine = HB;
    auto advance = [&](bool last, bool post) {
      ic += 8;
      iaddr += 128;
      if (__ballot(last) != 0) {  // some group moves to its next job
        const uint32_t s = gsrc + min(ik + 1, 7u);
        const uint32_t np = lane_get(jp, s), nnb = lane_get(jnb, s);
        const uint32_t nlo = lane_get(jlo, s), nhi = lane_get(jhi, s);
        const uint32_t nlim = post ? lane_get(lim_mine, np) : 0u;
        if (last) {
          ++ik;
          ip = np;
          inb_ = ik < 8u ? nnb : 0u;
          ic = gj;
          iaddr = ((uint64_t)nhi << 32 | nlo) + gj * 16u;
          ilim = nlim;
        }
      }
    };
    auto issue_pre = [&](int u) {
      const bool live = ic < inb_;
      glds<OO_RX_BODY_AUX>(live ? iaddr : dummy, &L.ring[u][0]);
      const bool last = inb_ != 0 && ic - gj + 8 >= inb_;
      meta[u] = ip | (ic << 6) | (live ? M_LIVE : 0u) | (last ? M_LAST : 0u);
      advance(last, false);
    };
    auto issue = [&](int u) {
      const bool live = ic < inb_;
      glds<OO_RX_BODY_AUX>(live ? iaddr : dummy, &L.ring[u][0]);
      const bool last = inb_ != 0 && ic - gj + 8 >= inb_;
      const int nv = live ? min(max((int)ilim - (HB + 16 * (int)ic), 0), 16) : 0;
      meta[u] = (uint32_t)nv | (last ? M_LAST : 0u);
      advance(last, true);
    };

    // Body prologue (lands during the parse), then wait for the header window.
#ifdef OO_RX_EXP_LATEPRO
    if (false) {
#else
    if (T >= (uint32_t)R) {
#endif
#pragma unroll
      for (int u = 0; u < R; ++u) issue_pre(u);
      vm_wait<R>();
    } else {
#pragma unroll
      for (int u = 0; u < R; ++u) {
        if ((uint32_t)u < T) issue_pre(u);
        else meta[u] = 0;
      }
      vm_wait<0>();
    }
    STAMP(1, __builtin_amdgcn_s_memrealtime());
    STAMP(7, T);

    const uint8_t* my = reinterpret_cast<const uint8_t*>(&L.hdr[0][lane]);
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

#ifdef OO_RX_EXP_STREAMONLY
    // Experiment build: no parse/demux; every frame's bytes past the window
    // are summed (timing of the stream machinery alone; records are garbage).
    oo_gpu_rx_result r;
    __builtin_memset(&r, 0, sizeof(r));
    const bool longl4 = span > HB;
    const int E4 = span;
    uint32_t s4 = 0, pseudo = 1;
    const uint32_t proto = 17, flags = 0;
#else
    // ---- 4. parse (per lane)
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
    // waits for the body stream (step 5) and the record below is speculative.
    const bool longl4 = reason == PENDING && need_l4 && E4 > HB;
    if (reason == PENDING && need_l4 && !longl4) {
      uint32_t f = fold16(s4);
      if (shift & 1) f = swap16(f);  // RFC 1071 byte-order swap
      if (fold16(f + pseudo) != 0xffffu)
        reason = proto == 6u ? OO_RX_R_TCP_CSUM : OO_RX_R_UDP_CSUM;
    }

    STAMP(2, __builtin_amdgcn_s_memrealtime());
    // ---- handle_rx_pkt, demux, record (per lane; netif_event.c:250-451).
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
        // Every stage's first slot bit, its successor's bit and the first
        // slot's record are loaded up front (two dependent levels); the walks
        // then usually need nothing more.
        if (is6) {
          const uint32_t zero[4] = {0, 0, 0, 0};
          const uint32_t dx = r.daddr_be, sx = r.saddr_be;
          const uint32_t mask = P.ip6_mask;
          const uint32_t h1_0 = hash3(dx, dport, sx, sport, proto) & mask;
          const uint32_t h1_1 = hash3(dx, dport, 0u, 0u, proto) & mask;
          const uint32_t h1_2 = hash3(0u, dport, 0u, 0u, proto) & mask;
          const uint32_t h2_0 = hash2(dx, dport, sx, sport, proto);
          const uint32_t h2_1 = hash2(dx, dport, 0u, 0u, proto);
          const uint32_t h2_2 = hash2(0u, dport, 0u, 0u, proto);
          const bool o0 = occ_bit(P.occ6, h1_0), o1 = occ_bit(P.occ6, h1_1);
          const bool o2 = nst == 3 && occ_bit(P.occ6, h1_2);
          const bool q0 = occ_bit(P.occ6, (h1_0 + h2_0) & mask);
          const bool q1 = occ_bit(P.occ6, (h1_1 + h2_1) & mask);
          const bool q2 = nst == 3 && occ_bit(P.occ6, (h1_2 + h2_2) & mask);
          Slot6 s0 = {}, s1 = {}, s2 = {};
          if (o0) s0 = load_slot6(P, h1_0);
          if (o1) s1 = load_slot6(P, h1_1);
          if (o2) s2 = load_slot6(P, h1_2);
          m = walk6(P, a6d, dport, a6s, false, sport, proto, intf_i, vlan, h1_0, h2_0, o0, s0, q0);
          stage = 1;
          if (m.n == 0) {
            m = walk6(P, a6d, dport, zero, true, 0u, proto, intf_i, vlan, h1_1, h2_1, o1, s1, q1);
            stage = 2;
          }
          if (m.n == 0 && nst == 3) {
            m = walk6(P, zero, dport, zero, true, 0u, proto, intf_i, vlan, h1_2, h2_2, o2, s2, q2);
            stage = 3;
          }
        } else {
          const uint32_t da = r.daddr_be, sa = r.saddr_be;
          const uint32_t mask = P.ip4_mask;
          const uint32_t h1_0 = hash3(da, dport, sa, sport, proto) & mask;
          const uint32_t h1_1 = hash3(da, dport, 0u, 0u, proto) & mask;
          const uint32_t h1_2 = hash3(0u, dport, 0u, 0u, proto) & mask;
          const uint32_t h2_0 = hash2(da, dport, sa, sport, proto);
          const uint32_t h2_1 = hash2(da, dport, 0u, 0u, proto);
          const uint32_t h2_2 = hash2(0u, dport, 0u, 0u, proto);
          const bool o0 = occ_bit(P.occ4, h1_0), o1 = occ_bit(P.occ4, h1_1);
          const bool o2 = nst == 3 && occ_bit(P.occ4, h1_2);
          const bool q0 = occ_bit(P.occ4, (h1_0 + h2_0) & mask);
          const bool q1 = occ_bit(P.occ4, (h1_1 + h2_1) & mask);
          const bool q2 = nst == 3 && occ_bit(P.occ4, (h1_2 + h2_2) & mask);
          Slot4 s0 = {}, s1 = {}, s2 = {};
          if (o0) s0 = load_slot4(P, h1_0);
          if (o1) s1 = load_slot4(P, h1_1);
          if (o2) s2 = load_slot4(P, h1_2);
          m = walk4(P, da, dport, sa, sport, proto, intf_i, vlan, h1_0, h2_0, o0, s0, q0);
          stage = 1;
          if (m.n == 0) {
            m = walk4(P, da, dport, 0u, 0u, proto, intf_i, vlan, h1_1, h2_1, o1, s1, q1);
            stage = 2;
          }
          if (m.n == 0 && nst == 3) {
            m = walk4(P, 0u, dport, 0u, 0u, proto, intf_i, vlan, h1_2, h2_2, o2, s2, q2);
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
#endif



    // ---- 5. body stream.  Each lane sums its chunk, masked at the L4 region
    // end (lim of its packet); on a group's last round of a packet the 8-lane
    // total goes to lane (g, job number), whose packet lane collects it
    // below.  Packets whose verdict is already final sum nothing (lim = HB).
#ifdef OO_RX_EXP_LATEPRO
#pragma unroll
    for (int u = 0; u < R; ++u) {
      if ((uint32_t)u < T) issue_pre(u);
      else meta[u] = 0;
    }
#endif
    lim_mine = longl4 ? (uint32_t)E4 : (uint32_t)HB;
    ilim = lane_get(lim_mine, ip);
#pragma unroll
    for (int u = 0; u < R; ++u) {  // the prologue's meta, now that lim is known
      const uint32_t mt = meta[u];
      const int lim = (int)lane_get(lim_mine, mt & 63u);
      const int nv = min(max(lim - (HB + 16 * (int)((mt >> 6) & 1023u)), 0), 16);
      meta[u] = (mt & M_LIVE ? (uint32_t)nv : 0u) | (mt & M_LAST);
    }
    uint32_t acc = 0, bs = 0, ck = 0;
    auto consume = [&](int u) {
      const uint32_t mt = meta[u];
      const uint4 v = lds_read16(&L.ring[u][lane]);
      const int nv = (int)(mt & 31u);
      if (nv == 16) acc = chunk_sum_all(v, acc);
      else if (nv != 0) acc += chunk_sum(v, 0, 0, nv);
      if (__ballot((mt & M_LAST) != 0) != 0) {
        const uint32_t t = group_sum8(acc);
        if (mt & M_LAST) {
          if (gj == ck) bs = t;
          ++ck;
          acc = 0;
        }
      }
    };
    STAMP(3, __builtin_amdgcn_s_memrealtime());
    for (uint32_t k0 = 0; k0 < T; k0 += R) {
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const uint32_t k = k0 + (uint32_t)u;
        if (k < T) {
          // Pieces k+1 .. min(T, k+R)-1 may still be in flight.
          if (k + R <= T) vm_wait<R - 1>();
          else vm_wait<0>();
          consume(u);
          if (k + R < T) issue(u);  // slot u was read (lds_read16 waited)
        }
      }
    }
    const uint32_t body = lane_get(bs, myslot);
    STAMP(4, __builtin_amdgcn_s_memrealtime());

    if (longl4) {
      // The verdict the speculative record waited for; a failure turns it
      // into the drop record (only the fields a drop defines survive).
      s4 += body;
      uint32_t f = fold16(s4);
      if (shift & 1) f = swap16(f);
      if (fold16(f + pseudo) != 0xffffu) {
        r.reason = (uint8_t)(proto == 6u ? OO_RX_R_TCP_CSUM : OO_RX_R_UDP_CSUM);
        r.flags = (uint8_t)(flags & (OO_RX_F_VLAN | OO_RX_F_IP6));
        r.stage = 0; r.l4_off = 0; r.sport_be = 0; r.dport_be = 0; r.nmatch = 0;
        r.saddr_be = 0; r.daddr_be = 0; r.sock = -1; r.hash3 = 0;
      }
    }

    if (valid) {
      atomicAdd(&ctr[r.reason & (OO_RX_R_COUNT - 1)], 1u);
      uint4* o = reinterpret_cast<uint4*>(P.out + idx);
      const uint4* src = reinterpret_cast<const uint4*>(&r);
      o[0] = src[0];
      o[1] = src[1];
    }
    STAMP(5, __builtin_amdgcn_s_memrealtime());
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
