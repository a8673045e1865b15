// SPDX-License-Identifier: BSD-2-Clause
//
// oo_rx_device.h -- layouts shared by the gfx950 kernels (oo_rx_kernel.hip)
// and the host side of the C ABI (oo_gpu_rx.cpp).  Internal; not installed.
#ifndef OO_RX_DEVICE_H
#define OO_RX_DEVICE_H

#include <stddef.h>
#include <stdint.h>

#include "../../include/oo_gpu_rx.h"

#ifdef __HIPCC__
#define OO_HD __host__ __device__ __forceinline__
#else
#define OO_HD inline
#endif

namespace oo_rx {

// Filter-table entry states (netif_table.c:34-42): IPv4 entries keep the
// socket id in the low 30 bits and the state in the top two.
constexpr uint32_t ST_MASK = 0xc0000000u;
constexpr uint32_t ID_MASK = 0x3fffffffu;
constexpr uint32_t ST_PREFERRED = 0x00000000u;
constexpr uint32_t ST_REHASHED = 0x40000000u;
constexpr uint32_t ST_EMPTY = 0x80000000u;
constexpr uint32_t ST_TOMBSTONE = 0xc0000000u;
// IPv6 entries: id >= 0 occupied (netif_table_ip6.c:10-11).
constexpr int32_t ID6_TOMBSTONE = -1;
constexpr int32_t ID6_EMPTY = -2;

OO_HD bool occupied(uint32_t st) { return ((~st) & ST_EMPTY & ST_TOMBSTONE) != 0; }

// __onload_hash3 / __onload_hash2 (src/include/onload/hash.h:84-93,
// 165-173) on network-order values held in host integers (little-endian).
OO_HD uint32_t hash3(uint32_t la, uint32_t lp, uint32_t ra, uint32_t rp, uint32_t proto) {
  uint32_t h = __builtin_bswap32(ra) ^ la ^ ((rp << 16) | lp) ^ proto;
  h ^= h >> 16;
  h ^= h >> 8;
  return h;
}
OO_HD uint32_t hash2(uint32_t la, uint32_t lp, uint32_t ra, uint32_t rp, uint32_t proto) {
  return ((la ^ ra) ^ ((lp << 16) | rp) ^ proto) | 1u;
}

// Host mirror of the IPv6 filter table entry
// ci_ip6_netif_filter_table_entry {id, route_count, laddr[16]}
// (ip_shared_types.h:579-583).
struct Ip6Entry {
  int32_t id;
  int32_t route_count;
  uint32_t laddr[4];
};
static_assert(sizeof(Ip6Entry) == 24, "ip6 entry layout");
static_assert(sizeof(oo_gpu_rx_sock) == 48, "socket record layout");
static_assert(sizeof(oo_gpu_rx_result) == 32, "result record layout");
static_assert(sizeof(oo_gpu_pkt_desc) == 16, "descriptor layout");

// Device copy of the filter tables, laid out for the probe (DESIGN.md
// "Filter tables in HBM").  Per visited slot the reference walk reads the
// table entry, the ext entry (lport) and then, through the entry's id, the
// socket's raddr/rport/protocol/bind2dev fields (netif_table.c:192-319,
// netif_table_ip6.c:110-189).  Here each slot is one record that already
// carries the fields of the socket its id names, rebuilt by the host mirror
// whenever the slot or that socket changes, so a visited slot is one 32-B
// (IPv4) or 64-B (IPv6) load.  A bitmap of the slots that are not EMPTY
// (1 bit per slot: 8 KiB for 2^16 IPv4 slots) ends most walks -- every walk
// ends at its first EMPTY slot -- without touching the record array.
struct Slot4 {
  uint32_t id_state;  // entry: id (30 bits) | state (2 bits), netif_table.c:34-42
  uint32_t laddr;     // entry
  uint32_t raddr;     // socket: sock_raddr_be32
  uint16_t lport;     // ext entry
  uint16_t rport;     // socket: sock_rport_be16
  uint8_t proto;      // socket: sock_protocol
  uint8_t rsvd0;
  uint16_t sflags;    // socket: OO_GPU_RX_SOCK_*
  int16_t b2d_vlan;   // socket: rx_bind2dev_vlan
  uint16_t rsvd1;
  uint64_t hwports;   // socket: rx_bind2dev_hwports
};
static_assert(sizeof(Slot4) == 32, "v4 slot record layout");

struct Slot6 {
  int32_t id;         // entry: >= 0 occupied, -1 tombstone, -2 empty
  int32_t route_count;  // entry
  uint32_t laddr[4];  // entry
  uint32_t raddr[4];  // socket: sock_ip6_raddr
  uint16_t lport;     // socket: sock_lport_be16
  uint16_t rport;     // socket: sock_rport_be16
  uint8_t proto;      // socket: sock_protocol
  uint8_t rsvd1;
  uint16_t sflags;    // socket: OO_GPU_RX_SOCK_*
  int16_t b2d_vlan;   // socket: rx_bind2dev_vlan
  uint16_t rsvd2;
  uint32_t rsvd3;
  uint64_t hwports;   // socket: rx_bind2dev_hwports
};
static_assert(sizeof(Slot6) == 64, "v6 slot record layout");

// One filter-table change, applied on the device in order by table_ops
// (oo_table_kernel.hip) -- the device side of ci_netif_filter_insert /
// _remove (netif_table.c:323-505, netif_table_ip6.c:192-345) and of a
// socket-field update.  64 bytes.
enum : uint8_t { OP_INSERT = 1, OP_REMOVE = 2, OP_SOCK = 3 };
struct TableOp {
  uint8_t kind;     // OP_*
  uint8_t af;       // 4 or 6 (INSERT / REMOVE)
  uint8_t proto;
  uint8_t rsvd0;
  uint16_t lport;   // network order
  uint16_t rport;
  int32_t sock;     // socket id
  uint32_t rsvd1;
  union {
    struct {
      uint32_t la[4];  // laddr (IPv4: la[0])
      uint32_t ra[4];  // raddr, zero for the wildcard
    } t;
    oo_gpu_rx_sock s;  // OP_SOCK
  } u;
};
static_assert(sizeof(TableOp) == 64, "table op layout");

// The key index (DESIGN.md "The key index"): the answer of every lookup key
// that has one, rebuilt on the device after each table change
// (oo_table_kernel.hip table_kx).  A lookup is then one load level instead
// of a walk along Onload's probe sequence.  Keys are a stage's lookup tuple;
// the value is the socket id of the walk's first match, with KX_FB when the
// walk's answer depends on the packet (a bind2dev socket among the matches)
// or its match count is not 1 (UDP) -- those lanes walk the table.
//  IPv4: two regions (UDP, then TCP) of kx_nb4 + KX_PAD4 buckets, a bucket
//   two 16-B entries {laddr, raddr, lport | rport << 16, value}.
//  IPv6: kx_ne6 + KX_PAD6 entries of 64 B {laddr[4], raddr[4],
//   lport | rport << 16, proto | wildcard << 8, value, 0 x 5}; a wildcard key
//   (raddr and rport zero) is a lookup with ra_null: unconnected sockets.
// A key is placed at its hash's bucket (entry) or the first free one after
// it, never wrapping: the last KX_OVF are overflow room, the pad after them
// always empty (a two-bucket load at the end reads it).  Value 0: empty.
constexpr uint32_t KX_VALID = 0x80000000u;
constexpr uint32_t KX_FB = 0x40000000u;
// A key that lost its last match since the index was built keeps its entry
// with this value (incremental maintenance, oo_table_kernel.hip): a lookup
// that meets it walks the table, and an entry never turns empty between two
// rebuilds, so no key's run gains an empty entry before the key.
constexpr uint32_t KX_DEAD = KX_FB;
// TableOp::rsvd0 bits set by the host for an incremental flush: the op owns
// the recomputation of its exact key / (IPv6) its wildcard key (one op per
// distinct key of the flush).
constexpr uint8_t KX_OWN_EXACT = 1, KX_OWN_WILD = 2;
constexpr uint32_t KX_OVF = 64;
constexpr uint32_t KX_PAD4 = KX_OVF + 2, KX_PAD6 = KX_OVF + 1;
constexpr uint32_t KX_WALK_MAX = 4096;  // a longer build walk turns the index off

OO_HD uint32_t kx_mix(uint32_t h) {
  h ^= h >> 16;
  h *= 0x7feb352du;
  h ^= h >> 15;
  h *= 0x846ca68bu;
  h ^= h >> 16;
  return h;
}
// The key hash: IPv4 keys with la[1..3] = ra[1..3] = 0 and pw = 0.  Each
// word's high half is folded into its low half before the multiply: the
// words hold network-order bytes, so a key's varying octets (the peer's last
// address byte, the ports) sit in the high bits, which a multiply never
// carries down -- without the fold, config 5's 4,160 TCP keys shared a home
// bucket 12x as often as random keys would (tools/kx_probe.py).
OO_HD uint32_t kx_fold(uint32_t w) { return w ^ (w >> 16); }
OO_HD uint32_t kx_hash(uint32_t la0, uint32_t la1, uint32_t la2, uint32_t la3, uint32_t ra0,
                       uint32_t ra1, uint32_t ra2, uint32_t ra3, uint32_t ports, uint32_t pw) {
  return kx_mix(kx_fold(la0) * 0x9e3779b1u + kx_fold(la1) * 0x85ebca77u + kx_fold(la2) * 0xc2b2ae3du +
                kx_fold(la3) * 0x27d4eb2fu + kx_fold(ra0) * 0x165667b1u + kx_fold(ra1) * 0xd3a2646du +
                kx_fold(ra2) * 0xfd7046c5u + kx_fold(ra3) * 0xb55a4f09u + kx_fold(ports) * 0x2545f491u +
                kx_fold(pw) * 0x9e3779b9u);
}

// Device-resident filter-table state of a context.
struct DevTables {
  Slot4* slot4;
  int32_t* rc4;       // route counts of the IPv4 slots (the ext entries)
  uint32_t* occ4;     // bit i: IPv4 slot i is not EMPTY
  Slot6* slot6;
  uint32_t* occ6;
  oo_gpu_rx_sock* socks;
  uint32_t* sockgen;  // flush generation of each socket's last change
  uint32_t ip4_mask, ip6_mask, max_socks;
  // The key index (null: none).
  uint32_t* kx4;
  uint32_t* kx6;
  uint32_t* kx_ok;    // 1: the index answers lookups (0: walks only)
  uint32_t kx_nb4;    // main IPv4 buckets per protocol region (a power of two)
  uint32_t kx_ne6;    // main IPv6 entries (a power of two)
};

// The zero region read by lanes that have no chunk to load (64 KiB, so
// those reads spread over the L2 channels).  The same allocation holds the
// sink (64 x 32 B) and the context's intf_i_to_hwport table after it.
constexpr uint32_t ZERO_LINES = 4096;
constexpr uint32_t SINK_BYTES = 64u * 32u;

// Wave groups of a launch at most: each has a tile-claim counter on a
// 128-B line of its own (KParams::claim).
constexpr uint32_t CLAIM_GROUPS = 64;
// One claim set: the window (or tile) kernel's group counters, the body
// kernel's group counters, and the body flag, each on a 128-B line.
constexpr uint32_t CLAIM_LINES = 2 * CLAIM_GROUPS + 1;

// A win_kernel block's copy of the occupancy bitmaps: the IPv4 bitmap at 0,
// the IPv6 one at OCC_LDS_B6, the intf -> hwport bytes at OCC_LDS_HW.  Tables
// of up to 2^16 IPv4 / 2^14 IPv6 slots (the defaults) fit; larger ones take
// the single-kernel path.
constexpr uint32_t OCC_LDS_B6 = 8192;
constexpr uint32_t OCC_LDS_HW = 8192 + 2048;
constexpr uint32_t OCC_LDS_BYTES = OCC_LDS_HW + 32;
constexpr uint32_t OCC_LDS_MAX4 = 1u << 16, OCC_LDS_MAX6 = 1u << 14;
constexpr uint32_t FLAG_LINE = 2 * CLAIM_GROUPS;
// The staged header window per packet (oo_rx_kernel.hip HB).
constexpr uint32_t HB_BYTES = 128;

// The split transform's pending word of a frame with a body (KParams::pend,
// 8 B per packet, written by win_kernel, read by body_kernel):
//  bits  0-15  the body-sum residue mod 0xffff for which the L4 checksum
//              passes; PEND_NONE: the verdict does not wait for the body
//  bit  16     TCP (else UDP)
//  bits 17-18  the record's OO_RX_F_IP6 / OO_RX_F_VLAN flags
//  bits 24-28  the record's reason as written (the sum passing)
//  bits 32-47  vlan, 48-63 ip_paylen (the drop record keeps them)
constexpr uint32_t PEND_NONE = 0xffffu;

// Kernel arguments (passed by value).
struct KParams {
  const uint8_t* frames;
  uint64_t frames_bytes;
  const oo_gpu_pkt_desc* desc;  // or struct xdp_desc[ring_mask + 1] (xdp)
  uint32_t ring_mask;    // descriptor i is desc[(ring_cons + i) & ring_mask]
  uint32_t ring_cons;    // (~0u and 0 for a plain descriptor array)
  uint32_t xdp;          // 1: AF_XDP ring entries {u64 addr; u32 len; u32 options}
  int32_t xdp_intf;      // the ring's interface (xdp)
  oo_gpu_rx_result* out;
  uint32_t* counters;  // OO_RX_R_COUNT u32, may be null
  uint32_t n;
  uint32_t ntiles;  // tiles (oo_rx_kernel.hip "Tiles")
  uint32_t tlo;     // tile sizes: tlo + tstep for tiles < ta, else tlo (the last: the rest)
  uint32_t ta;
  uint32_t tstep;   // 8 (job slots fill), or 1 (OO_RX_TSTEP=1: sizes within one packet)
  uint32_t ip4_mask;
  uint32_t ip6_mask;
  const Slot4* slot4;
  const uint32_t* occ4;  // bit i set: IPv4 slot i is not EMPTY
  const Slot6* slot6;
  const uint32_t* occ6;  // bit i set: IPv6 slot i is not EMPTY
  const uint8_t* zero;   // ZERO_LINES x 16 B of zeros (lanes with nothing to read)
  uint8_t* sink;         // 64 x 32 B written by lanes without a packet (rx_kernel)
  uint64_t* stamps;      // diagnostic builds (OO_RX_STAMPS) only; may be null
  uint32_t* claim;       // one counter per wave group, 128 B apart, 0 at launch
  uint32_t* claim_next;  // the set the stream's next launch claims from: zeroed here
  uint32_t ngroups;      // wave groups (a power of two, ngroups << gshift <= waves)
  uint32_t gshift;       // wave gwave is in group (gwave >> gshift) mod ngroups
  uint32_t dyn;          // 1: tiles past a wave's first three are claimed
  const uint8_t* hwport;  // intf_i_to_hwport, OO_GPU_RX_MAX_INTF bytes in device memory
  uint64_t* pend;        // split transform: a pending word per packet (n + 64 entries)
  uint32_t* flag;        // split transform: non-zero once a verdict waits for a body
  // The key index (DevTables kx*); kx4 null: lookups walk the tables.
  const uint32_t* kx4;
  const uint32_t* kx6;
  const uint32_t* kx_ok;
  uint32_t kx_nb4, kx_ne6;
};

// The poll instance's kernel arguments (oo_rx_kernel.hip "The poll
// instance"): the batch's KParams and its completion (done null: none).
struct PollArgs {
  KParams P;
  uint32_t* done_ctr;  // the launch's claim-set FLAG_LINE word (0 at launch)
  uint32_t* done;      // host-mapped word: done_val once every record has landed
  uint32_t done_val;
  uint32_t rsvd;
};

}  // namespace oo_rx

#endif
