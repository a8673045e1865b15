// SPDX-License-Identifier: BSD-2-Clause
//
// oo_table_kernel.hip -- device-side filter-table maintenance (SURVEY.md
// §8(f) row 4): the oof-driven filter inserts and removes
// (src/lib/efthrm/oof_interface.c:184-262 -> ci_netif_filter_insert /
// _remove) applied to the HBM copy of the tables on the batch stream, in
// the order the stack lock saw them, with no host synchronisation.
//
//   ci_ip4_netif_filter_insert    src/lib/transport/ip/netif_table.c:323-406
//   __ci_ip4_netif_filter_remove  netif_table.c:409-443
//   ci_ip4_netif_filter_remove    netif_table.c:447-495
//   ci_ip6_netif_filter_insert    src/lib/transport/ip/netif_table_ip6.c:192-262
//   ci_ip6_netif_filter_remove    netif_table_ip6.c:264-345
//
// The host keeps its own mirror (oo_gpu_rx.cpp) for the calls that return
// at once (insert's -ENOBUFS, exact lookups); both apply the same ops in the
// same order, so the HBM tables equal the mirror slot for slot -- route
// counts and tombstones included (tests/test_gpu_tables.py).
//
// The device slot records (oo_rx_device.h Slot4 / Slot6) also carry the
// fields of the socket each slot's id names.  A socket change (OP_SOCK)
// marks the socket with the flush generation; table_refresh then rewrites
// every slot that names a marked socket -- an O(table) pass, but a GPU one
// (2^16 + 2^14 slots) on the stream, not a host rescan.
//
// The ops of a flush arrive in levels (oo_gpu_rx.cpp push_op): the ops of
// one level touch disjoint slots -- the probe walks the host mirror did for
// them -- so they commute, and table_ops applies a level one op per lane,
// the levels in order with a workgroup barrier between them.  Socket-field
// ops are all level 0 (one per socket: the last change wins), and the
// refresh pass that follows rewrites every slot of a changed socket, so
// when an insert reads a socket's fields does not matter.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "oo_rx_device.h"

namespace oo_rx {

// Ops of one level touch disjoint slots but may share an occupancy word.
__device__ __forceinline__ void occ_set(uint32_t* occ, uint32_t i, bool on) {
  const uint32_t b = 1u << (i & 31u);
  if (on)
    atomicOr(&occ[i >> 5], b);
  else
    atomicAnd(&occ[i >> 5], ~b);
}

// The socket fields of slot records (what netif_table.c:192-231 reads through
// an entry's id).
__device__ __forceinline__ void slot4_sock(Slot4& r, const oo_gpu_rx_sock& k) {
  r.raddr = k.raddr_be32;
  r.rport = k.rport_be16;
  r.proto = k.protocol;
  r.sflags = k.flags;
  r.b2d_vlan = k.bind2dev_vlan;
  r.hwports = k.bind2dev_hwports;
}
__device__ __forceinline__ void slot4_nosock(Slot4& r) {
  r.raddr = 0;
  r.rport = 0;
  r.proto = 0;
  r.sflags = 0;
  r.b2d_vlan = 0;
  r.hwports = 0;
}
__device__ __forceinline__ void slot6_sock(Slot6& r, const oo_gpu_rx_sock& k) {
  for (int i = 0; i < 4; ++i) {
    uint32_t w;
    __builtin_memcpy(&w, k.raddr6 + 4 * i, 4);
    r.raddr[i] = w;
  }
  r.lport = k.lport_be16;
  r.rport = k.rport_be16;
  r.proto = k.protocol;
  r.sflags = k.flags;
  r.b2d_vlan = k.bind2dev_vlan;
  r.hwports = k.bind2dev_hwports;
}
__device__ __forceinline__ void slot6_nosock(Slot6& r) {
  for (int i = 0; i < 4; ++i) r.raddr[i] = 0;
  r.lport = 0;
  r.rport = 0;
  r.proto = 0;
  r.sflags = 0;
  r.b2d_vlan = 0;
  r.hwports = 0;
}

// ci_ip4_netif_filter_insert: route counts of the occupied slots passed are
// raised (and stay raised when the table is full, :349-376).
__device__ void ip4_insert(const DevTables& T, const TableOp& op) {
  const uint32_t la = op.u.t.la[0], ra = op.u.t.ra[0];
  uint32_t h1 = hash3(la, op.lport, ra, op.rport, op.proto) & T.ip4_mask;
  const uint32_t h2 = hash2(la, op.lport, ra, op.rport, op.proto);
  const uint32_t first = h1;
  while (occupied(T.slot4[h1].id_state)) {
    ++T.rc4[h1];
    h1 = (h1 + h2) & T.ip4_mask;
    if (h1 == first) return;  // -ENOBUFS (the host mirror reports it)
  }
  Slot4 r = T.slot4[h1];
  r.id_state = (h1 == first ? ST_PREFERRED : ST_REHASHED) | ((uint32_t)op.sock & ID_MASK);
  r.laddr = la;
  r.lport = op.lport;
  slot4_sock(r, T.socks[op.sock]);
  T.slot4[h1] = r;
  occ_set(T.occ4, h1, true);
}

// ci_ip4_netif_filter_remove + __ci_ip4_netif_filter_remove.
__device__ void ip4_remove(const DevTables& T, const TableOp& op) {
  const uint32_t la = op.u.t.la[0], ra = op.u.t.ra[0];
  const uint32_t h1 = hash3(la, op.lport, ra, op.rport, op.proto) & T.ip4_mask;
  const uint32_t h2 = hash2(la, op.lport, ra, op.rport, op.proto);
  const uint32_t id = (uint32_t)op.sock & ID_MASK;
  uint32_t i = h1;
  int hops = 0;
  for (;;) {
    const uint32_t st = T.slot4[i].id_state;
    if (occupied(st) && (st & ID_MASK) == id) {
      if (T.slot4[i].laddr == la) break;
    } else if ((st & ST_MASK) == ST_EMPTY) {
      return;  // removes of an absent filter are allowed (:476-481)
    }
    i = (i + h2) & T.ip4_mask;
    ++hops;
    if (i == h1) return;
  }
  auto to_empty = [&](uint32_t k) {
    Slot4 r = T.slot4[k];
    r.id_state = (r.id_state & ID_MASK) | ST_EMPTY;
    slot4_nosock(r);
    T.slot4[k] = r;
    occ_set(T.occ4, k, false);
  };
  i = h1;
  for (int k = 0; k < hops; ++k) {
    if (--T.rc4[i] == 0 && (T.slot4[i].id_state & ST_MASK) == ST_TOMBSTONE) to_empty(i);
    i = (i + h2) & T.ip4_mask;
  }
  if (T.rc4[i] == 0) {
    to_empty(i);
  } else {
    T.slot4[i].id_state = (T.slot4[i].id_state & ID_MASK) | ST_TOMBSTONE;
  }
}

__device__ __forceinline__ uint32_t addr_xor4(const uint32_t a[4]) {
  return a[0] ^ a[1] ^ a[2] ^ a[3];
}

__device__ __forceinline__ bool laddr6_eq(const Slot6& r, const uint32_t a[4]) {
  return r.laddr[0] == a[0] && r.laddr[1] == a[1] && r.laddr[2] == a[2] && r.laddr[3] == a[3];
}

// ci_ip6_netif_filter_insert: the same walk over 24-B entries whose id is
// >= 0 when occupied.
__device__ void ip6_insert(const DevTables& T, const TableOp& op) {
  const uint32_t lx = addr_xor4(op.u.t.la), rx = addr_xor4(op.u.t.ra);
  uint32_t h1 = hash3(lx, op.lport, rx, op.rport, op.proto) & T.ip6_mask;
  const uint32_t h2 = hash2(lx, op.lport, rx, op.rport, op.proto);
  const uint32_t first = h1;
  while (T.slot6[h1].id >= 0) {
    ++T.slot6[h1].route_count;
    h1 = (h1 + h2) & T.ip6_mask;
    if (h1 == first) return;  // -ENOBUFS
  }
  Slot6 r = T.slot6[h1];
  r.id = op.sock;
  for (int k = 0; k < 4; ++k) r.laddr[k] = op.u.t.la[k];
  slot6_sock(r, T.socks[op.sock]);
  T.slot6[h1] = r;
  occ_set(T.occ6, h1, true);
}

// ci_ip6_netif_filter_remove: a tombstone loses its id (-1).
__device__ void ip6_remove(const DevTables& T, const TableOp& op) {
  const uint32_t lx = addr_xor4(op.u.t.la), rx = addr_xor4(op.u.t.ra);
  const uint32_t h1 = hash3(lx, op.lport, rx, op.rport, op.proto) & T.ip6_mask;
  const uint32_t h2 = hash2(lx, op.lport, rx, op.rport, op.proto);
  uint32_t i = h1;
  int hops = 0;
  for (;;) {
    const int32_t id = T.slot6[i].id;
    if (id == op.sock) {
      if (laddr6_eq(T.slot6[i], op.u.t.la)) break;
    } else if (id == ID6_EMPTY) {
      return;
    }
    i = (i + h2) & T.ip6_mask;
    ++hops;
    if (i == h1) return;
  }
  auto set_id = [&](uint32_t k, int32_t nid) {
    Slot6 r = T.slot6[k];
    r.id = nid;
    slot6_nosock(r);
    T.slot6[k] = r;
    occ_set(T.occ6, k, nid != ID6_EMPTY);
  };
  i = h1;
  for (int k = 0; k < hops; ++k) {
    if (--T.slot6[i].route_count == 0 && T.slot6[i].id == ID6_TOMBSTONE) set_id(i, ID6_EMPTY);
    i = (i + h2) & T.ip6_mask;
  }
  set_id(i, T.slot6[i].route_count == 0 ? ID6_EMPTY : ID6_TOMBSTONE);
}

__device__ __forceinline__ void apply_op(const DevTables& T, const TableOp& op, uint32_t gen) {
  if (op.sock < 0 || (uint32_t)op.sock >= T.max_socks) return;  // the host rejected it
  if (op.kind == OP_SOCK) {
    T.socks[op.sock] = op.u.s;
    T.sockgen[op.sock] = gen;
  } else if (op.kind == OP_INSERT) {
    if (op.af == 4) ip4_insert(T, op);
    else ip6_insert(T, op);
  } else if (op.kind == OP_REMOVE) {
    if (op.af == 4) ip4_remove(T, op);
    else ip6_remove(T, op);
  }  // kind 0: a socket op superseded by a later one
}

// Slots whose socket changed in flush `gen` take its new fields (IPv4: every
// slot that is not EMPTY keeps its id; IPv6: occupied slots).
__global__ __launch_bounds__(256) void table_refresh(DevTables T, uint32_t gen) {
  const uint32_t n4 = T.ip4_mask + 1u, n6 = T.ip6_mask + 1u;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n4 + n6;
       i += gridDim.x * blockDim.x) {
    if (i < n4) {
      const uint32_t st = T.slot4[i].id_state;
      const uint32_t id = st & ID_MASK;
      if ((st & ST_MASK) != ST_EMPTY && id < T.max_socks && T.sockgen[id] == gen) {
        Slot4 r = T.slot4[i];
        slot4_sock(r, T.socks[id]);
        T.slot4[i] = r;
      }
    } else {
      const uint32_t j = i - n4;
      const int32_t id = T.slot6[j].id;
      if (id >= 0 && (uint32_t)id < T.max_socks && T.sockgen[id] == gen) {
        Slot6 r = T.slot6[j];
        slot6_sock(r, T.socks[id]);
        T.slot6[j] = r;
      }
    }
  }
}

// Fresh tables: every slot EMPTY (netif_table.c:592-611: IPv4 state EMPTY,
// netif_table_ip6.c:349-365: id -2), no sockets, no occupancy.
__global__ __launch_bounds__(256) void table_init(DevTables T) {
  const uint32_t n4 = T.ip4_mask + 1u, n6 = T.ip6_mask + 1u;
  const uint32_t total = n4 + n6 + T.max_socks;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    if (i < n4) {
      Slot4 r = {};
      r.id_state = ST_EMPTY;
      T.slot4[i] = r;
      T.rc4[i] = 0;
      if ((i & 31u) == 0) T.occ4[i >> 5] = 0;
    } else if (i < n4 + n6) {
      const uint32_t j = i - n4;
      Slot6 r = {};
      r.id = ID6_EMPTY;
      T.slot6[j] = r;
      if ((j & 31u) == 0) T.occ6[j >> 5] = 0;
    } else {
      const uint32_t k = i - n4 - n6;
      T.socks[k] = oo_gpu_rx_sock{};
      T.sockgen[k] = 0;
    }
  }
}

// Occupancy bits from the slot records (after an image import).
__global__ __launch_bounds__(256) void table_occ(DevTables T) {
  const uint32_t w4 = (T.ip4_mask + 1u + 31u) >> 5, w6 = (T.ip6_mask + 1u + 31u) >> 5;
  for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < w4 + w6;
       w += gridDim.x * blockDim.x) {
    uint32_t bits = 0;
    if (w < w4) {
      for (uint32_t b = 0; b < 32u && w * 32u + b <= T.ip4_mask; ++b)
        if ((T.slot4[w * 32u + b].id_state & ST_MASK) != ST_EMPTY) bits |= 1u << b;
      T.occ4[w] = bits;
    } else {
      const uint32_t v = w - w4;
      for (uint32_t b = 0; b < 32u && v * 32u + b <= T.ip6_mask; ++b)
        if (T.slot6[v * 32u + b].id != ID6_EMPTY) bits |= 1u << b;
      T.occ6[v] = bits;
    }
  }
}

// ---------------------------------------------------------------------------
// The key index (oo_rx_device.h): one thread per slot.  A slot whose entry is
// the first match of its own key's walk -- the walk the RX kernels would do
// for a packet of that key, netif_table.c:234-319 / netif_table_ip6.c:110-189
// -- puts the key's answer into the index; every other key has no match, and
// finds no entry.  Keys are exact tuples: on IPv4 the first probe's unchecked
// lport is safe by the Local Port Recovery Property of tables of 2^16+ slots
// (netif_table.c:276-290), for entries at the slot their key hashes to; an
// entry left PREFERRED elsewhere (its socket's fields changed after the
// insert) turns the index off, as do a full overflow room and a walk longer
// than KX_WALK_MAX.

__device__ __forceinline__ void kx_off(const DevTables& T) { T.kx_ok[0] = 0u; }

struct KxWalk {
  uint32_t first;  // slot of the first match (~0u: none)
  uint32_t n;      // matches (TCP: stops at the first)
  bool b2d;        // a match is a bind2dev socket (its verdict depends on the packet)
  bool ok;         // false: walk too long
};

__device__ KxWalk kx_walk4(const DevTables& T, uint32_t la, uint32_t lp, uint32_t ra, uint32_t rp,
                           uint32_t proto) {
  KxWalk w = {~0u, 0u, false, true};
  const uint32_t first = hash3(la, lp, ra, rp, proto) & T.ip4_mask;
  const uint32_t h2 = hash2(la, lp, ra, rp, proto);
  uint32_t k = first;
  Slot4 e = T.slot4[k];
  auto hit = [&](uint32_t at, const Slot4& s) {
    if (w.n == 0) w.first = at;
    ++w.n;
    w.b2d |= (s.sflags & OO_GPU_RX_SOCK_BIND2DEV) != 0;
  };
  // the first probe: a PREFERRED entry, lport implied (netif_table.c:291-297)
  if ((e.id_state & ST_MASK) == ST_PREFERRED && e.laddr == la && e.raddr == ra && e.rport == rp &&
      e.proto == proto)
    hit(k, e);
  for (uint32_t steps = 0; !(proto == 6u && w.n != 0); ++steps) {
    if ((e.id_state & ST_MASK) == ST_EMPTY) break;
    k = (k + h2) & T.ip4_mask;
    if (k == first) break;
    if (steps >= KX_WALK_MAX) {
      w.ok = false;
      break;
    }
    e = T.slot4[k];
    if (occupied(e.id_state) && e.laddr == la && e.lport == lp && e.raddr == ra && e.rport == rp &&
        e.proto == proto)
      hit(k, e);
  }
  return w;
}

__device__ KxWalk kx_walk6(const DevTables& T, const uint32_t la[4], uint32_t lp,
                           const uint32_t ra[4], uint32_t rp, uint32_t proto, bool wild) {
  KxWalk w = {~0u, 0u, false, true};
  const uint32_t lx = addr_xor4(la), rx = wild ? 0u : addr_xor4(ra);
  const uint32_t first = hash3(lx, lp, rx, wild ? 0u : rp, proto) & T.ip6_mask;
  const uint32_t h2 = hash2(lx, lp, rx, wild ? 0u : rp, proto);
  uint32_t k = first;
  for (uint32_t steps = 0;; ++steps) {
    const Slot6 e = T.slot6[k];
    if (e.id == ID6_EMPTY) break;
    const bool rok = wild ? !(e.sflags & OO_GPU_RX_SOCK_CONNECTED)
                          : (e.raddr[0] == ra[0] && e.raddr[1] == ra[1] && e.raddr[2] == ra[2] &&
                             e.raddr[3] == ra[3] && e.rport == rp);
    if (e.id >= 0 && laddr6_eq(e, la) && e.lport == lp && e.proto == proto && rok) {
      if (w.n == 0) w.first = k;
      ++w.n;
      w.b2d |= (e.sflags & OO_GPU_RX_SOCK_BIND2DEV) != 0;
      if (proto == 6u) break;  // TCP: the first match ends the walk
    }
    k = (k + h2) & T.ip6_mask;
    if (k == first) break;
    if (steps >= KX_WALK_MAX) {
      w.ok = false;
      break;
    }
  }
  return w;
}

__device__ __forceinline__ uint32_t kx_value(const KxWalk& w, uint32_t id, uint32_t proto) {
  const bool fb = w.b2d || (proto == 17u && w.n != 1u);
  return KX_VALID | (fb ? KX_FB : 0u) | (id & ID_MASK);
}

// Claims the first free entry at or after the key's bucket (two entries of
// 16 B per bucket); false when the overflow room is full.
__device__ bool kx_put4(const DevTables& T, uint32_t proto, uint32_t la, uint32_t ra, uint32_t ports,
                        uint32_t val) {
  uint32_t* base = T.kx4 + (proto == 6u ? (size_t)(T.kx_nb4 + KX_PAD4) * 8u : 0u);
  const uint32_t b = kx_hash(la, 0, 0, 0, ra, 0, 0, 0, ports, 0) & (T.kx_nb4 - 1u);
  for (uint32_t q = b; q < T.kx_nb4 + KX_OVF; ++q) {
    for (uint32_t e = 0; e < 2; ++e) {
      uint32_t* ent = base + (size_t)q * 8u + e * 4u;
      if (atomicCAS(ent + 3, 0u, val) == 0u) {
        ent[0] = la;
        ent[1] = ra;
        ent[2] = ports;
        return true;
      }
    }
  }
  return false;
}

__device__ bool kx_put6(const DevTables& T, const uint32_t la[4], const uint32_t ra[4],
                        uint32_t ports, uint32_t pw, uint32_t val) {
  const uint32_t b = kx_hash(la[0], la[1], la[2], la[3], ra[0], ra[1], ra[2], ra[3], ports, pw) &
                     (T.kx_ne6 - 1u);
  for (uint32_t q = b; q < T.kx_ne6 + KX_OVF; ++q) {
    uint32_t* ent = T.kx6 + (size_t)q * 16u;
    if (atomicCAS(ent + 10, 0u, val) == 0u) {
      for (int i = 0; i < 4; ++i) {
        ent[i] = la[i];
        ent[4 + i] = ra[i];
      }
      ent[8] = ports;
      ent[9] = pw;
      return true;
    }
  }
  return false;
}

__global__ __launch_bounds__(256) void table_kx(DevTables T) {
  const uint32_t n4 = T.ip4_mask + 1u, n6 = T.ip6_mask + 1u;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n4 + n6;
       i += gridDim.x * blockDim.x) {
    if (i < n4) {
      const Slot4 r = T.slot4[i];
      const uint32_t st = r.id_state;
      const uint32_t id = st & ID_MASK;
      if (!occupied(st) || id >= T.max_socks || (r.proto != 6u && r.proto != 17u)) continue;
      if ((st & ST_MASK) == ST_PREFERRED &&
          (hash3(r.laddr, r.lport, r.raddr, r.rport, r.proto) & T.ip4_mask) != i) {
        kx_off(T);
        continue;
      }
      const KxWalk w = kx_walk4(T, r.laddr, r.lport, r.raddr, r.rport, r.proto);
      if (!w.ok) {
        kx_off(T);
      } else if (w.first == i &&
                 !kx_put4(T, r.proto, r.laddr, r.raddr, (uint32_t)r.lport | ((uint32_t)r.rport << 16),
                          kx_value(w, id, r.proto))) {
        kx_off(T);
      }
    } else {
      const uint32_t j = i - n4;
      const Slot6 r = T.slot6[j];
      if (r.id < 0 || (uint32_t)r.id >= T.max_socks || (r.proto != 6u && r.proto != 17u)) continue;
      const uint32_t zero[4] = {0, 0, 0, 0};
      // the exact tuple (stage 1), and for an unconnected socket the
      // wildcard (stages 2 and 3, ra_null)
      for (int wild = 0; wild < 2; ++wild) {
        if (wild && (r.sflags & OO_GPU_RX_SOCK_CONNECTED)) break;
        const KxWalk w = kx_walk6(T, r.laddr, r.lport, r.raddr, r.rport, r.proto, wild != 0);
        if (!w.ok) {
          kx_off(T);
        } else if (w.first == j &&
                   !kx_put6(T, r.laddr, wild ? zero : r.raddr,
                            (uint32_t)r.lport | (wild ? 0u : (uint32_t)r.rport << 16),
                            r.proto | (wild ? 0x100u : 0u), kx_value(w, (uint32_t)r.id, r.proto))) {
          kx_off(T);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Incremental key-index maintenance (a flush of filter ops only, one chunk,
// the index on).  After the flush's ops, the answers of the ops' own keys are
// walked again and written into the index; no other key's answer can have
// changed:
//  * a slot an insert fills was EMPTY or a tombstone.  A walk of another key
//    passes a filled tombstone as it passed the tombstone, and the new entry
//    is not that key's match (keys are exact tuples; the first probe's
//    unchecked lport is the Local Port Recovery Property's,
//    netif_table.c:276-290).  A walk that ended at the filled EMPTY slot had
//    no match past it: every entry past a slot on its key's probe sequence
//    raised that slot's route count when it went in (:349-376), so the slot
//    could not be EMPTY while such an entry was there.
//  * a remove turns the entry's slot, and passed tombstones whose route
//    count drops to 0, into tombstones or EMPTY slots; by the same count
//    argument no other key has a match past a slot that becomes EMPTY.
// Socket-field changes, ops whose tuple is not their socket's (the host
// checks both) and larger flushes take the full rebuild instead.
// A key that lost its last match keeps its entry as KX_DEAD (its lookups walk
// the table); an overflow, a long walk or an index that is already off asks
// the host for a full rebuild at the next flush (kx_req, host memory).

// The value word of the key's entry, or nullptr when the key has none (the
// first empty entry along its run ends the search, as it ends a lookup).
__device__ uint32_t* kx_find4(const DevTables& T, uint32_t proto, uint32_t la, uint32_t ra,
                              uint32_t ports) {
  uint32_t* base = T.kx4 + (proto == 6u ? (size_t)(T.kx_nb4 + KX_PAD4) * 8u : 0u);
  const uint32_t b = kx_hash(la, 0, 0, 0, ra, 0, 0, 0, ports, 0) & (T.kx_nb4 - 1u);
  for (uint32_t q = b; q < T.kx_nb4 + KX_OVF; ++q) {
    for (uint32_t e = 0; e < 2; ++e) {
      uint32_t* ent = base + (size_t)q * 8u + e * 4u;
      if (ent[3] == 0u) return nullptr;
      if (ent[0] == la && ent[1] == ra && ent[2] == ports) return ent + 3;
    }
  }
  return nullptr;
}

__device__ uint32_t* kx_find6(const DevTables& T, const uint32_t la[4], const uint32_t ra[4],
                              uint32_t ports, uint32_t pw) {
  const uint32_t b = kx_hash(la[0], la[1], la[2], la[3], ra[0], ra[1], ra[2], ra[3], ports, pw) &
                     (T.kx_ne6 - 1u);
  for (uint32_t q = b; q < T.kx_ne6 + KX_OVF; ++q) {
    uint32_t* ent = T.kx6 + (size_t)q * 16u;
    if (ent[10] == 0u) return nullptr;
    if (ent[0] == la[0] && ent[1] == la[1] && ent[2] == la[2] && ent[3] == la[3] &&
        ent[4] == ra[0] && ent[5] == ra[1] && ent[6] == ra[2] && ent[7] == ra[3] &&
        ent[8] == ports && ent[9] == pw)
      return ent + 10;
  }
  return nullptr;
}

// One index key an op owns, between the two phases.
struct KxKey {
  uint32_t la[4], ra[4], ports, pw, val;
  bool claim;  // phase 2: the key has no entry yet and a live answer
};

__device__ __forceinline__ void kx_request_full(uint32_t* kx_req) {
  __hip_atomic_store(kx_req, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Phase 1 for one key: its walk's answer, written in place when the key has
// an entry.
__device__ void kx_key_phase1(const DevTables& T, uint32_t af, uint32_t proto, bool wild,
                              KxKey& k, uint32_t* kx_req) {
  KxWalk w;
  uint32_t id = 0;
  uint32_t* at;
  if (af == 4) {
    w = kx_walk4(T, k.la[0], k.ports & 0xffffu, k.ra[0], k.ports >> 16, proto);
    if (w.n) id = T.slot4[w.first].id_state & ID_MASK;
  } else {
    w = kx_walk6(T, k.la, k.ports & 0xffffu, k.ra, k.ports >> 16, proto, wild);
    if (w.n) id = (uint32_t)T.slot6[w.first].id;
  }
  if (!w.ok) {
    kx_off(T);
    kx_request_full(kx_req);
    return;
  }
  k.val = w.n ? kx_value(w, id, proto) : KX_DEAD;
  at = af == 4 ? kx_find4(T, proto, k.la[0], k.ra[0], k.ports) : kx_find6(T, k.la, k.ra, k.ports, k.pw);
  if (at != nullptr) *at = k.val;  // (a dead key stays in place: lookups walk)
  else k.claim = w.n != 0;
}

// The ops of one flush chunk: level L is ops[lev_end[L-1], lev_end[L]).
// kx_mode 1: then the incremental index update for the ops (at most one per
// thread) that own a key.
constexpr int TABLE_THREADS = 1024;
__global__ __launch_bounds__(TABLE_THREADS) void table_ops(DevTables T, const TableOp* ops,
                                                           const uint32_t* lev_end, uint32_t nlev,
                                                           uint32_t gen, uint32_t kx_mode,
                                                           uint32_t* kx_req) {
  __shared__ uint32_t kx_on;
  if (kx_mode && threadIdx.x == 0) kx_on = T.kx_ok[0];
  uint32_t start = 0;
  for (uint32_t L = 0; L < nlev; ++L) {
    const uint32_t end = lev_end[L];
    for (uint32_t k = start + threadIdx.x; k < end; k += TABLE_THREADS) apply_op(T, ops[k], gen);
    __syncthreads();  // the next level sees this one's slots (and kx_on is set)
    start = end;
  }
  if (!kx_mode) return;
  __syncthreads();  // (kx_on, also for a chunk of no levels)
  if (kx_on == 0u) {  // off since the last rebuild: only a rebuild brings it back
    if (threadIdx.x == 0) kx_request_full(kx_req);
    return;
  }
  // Phase 1: every owned key's answer; keys with an entry are updated.
  KxKey key[2];
  uint32_t af = 0, proto = 0;
  key[0].claim = key[1].claim = false;
  if (threadIdx.x < start) {  // (start: the chunk's op count, at most TABLE_THREADS)
    const TableOp op = ops[threadIdx.x];
    af = op.af;
    proto = op.proto;
    if ((op.kind == OP_INSERT || op.kind == OP_REMOVE) && (proto == 6u || proto == 17u)) {
      for (int i = 0; i < 4; ++i) {
        key[0].la[i] = key[1].la[i] = af == 4 && i ? 0u : op.u.t.la[i];
        key[0].ra[i] = af == 4 && i ? 0u : op.u.t.ra[i];
        key[1].ra[i] = 0u;
      }
      key[0].ports = (uint32_t)op.lport | ((uint32_t)op.rport << 16);
      key[0].pw = af == 6 ? proto : 0u;
      key[1].ports = op.lport;
      key[1].pw = proto | 0x100u;
      if (op.rsvd0 & KX_OWN_EXACT) kx_key_phase1(T, af, proto, false, key[0], kx_req);
      if (af == 6 && (op.rsvd0 & KX_OWN_WILD)) kx_key_phase1(T, af, proto, true, key[1], kx_req);
    }
  }
  __syncthreads();  // every search is done before any claim writes a key
  // Phase 2: new keys claim the first free entry of their run.
  for (int j = 0; j < 2; ++j) {
    if (!key[j].claim) continue;
    const bool ok = af == 4 ? kx_put4(T, proto, key[j].la[0], key[j].ra[0], key[j].ports, key[j].val)
                            : kx_put6(T, key[j].la, key[j].ra, key[j].ports, key[j].pw, key[j].val);
    if (!ok) {
      kx_off(T);
      kx_request_full(kx_req);
    }
  }
}

// ---------------------------------------------------------------------------
// A batch's frame-length profile for the launch choice (oo_gpu_rx.cpp
// launch(): mixed sizes take the split transform): 256 descriptors evenly
// spaced over the batch (plain or AF_XDP ring entries: the length is the
// 16-bit field at byte 8 in both), their count, sum and sum of squares, stored
// to host memory with the sequence number last (the host reads it once the
// launch's event has completed).
__global__ __launch_bounds__(256) void len_sample(const uint8_t* desc, uint32_t n, uint32_t ring_mask,
                                                  uint32_t cons, uint32_t* out, uint32_t seq) {
  __shared__ uint64_t acc[3];
  const uint32_t t = threadIdx.x;
  if (t < 3u) acc[t] = 0;
  __syncthreads();
  if (n != 0 && (n >= 256u || t < n)) {
    const uint32_t i = n >= 256u ? (uint32_t)(((uint64_t)t * n) >> 8) : t;
    const uint32_t len = *reinterpret_cast<const uint16_t*>(desc + 16ull * ((cons + i) & ring_mask) + 8u);
    atomicAdd(reinterpret_cast<unsigned long long*>(&acc[0]), 1ull);
    atomicAdd(reinterpret_cast<unsigned long long*>(&acc[1]), (unsigned long long)len);
    atomicAdd(reinterpret_cast<unsigned long long*>(&acc[2]), (unsigned long long)len * len);
  }
  __syncthreads();
  if (t == 0) {
    for (int k = 0; k < 3; ++k) {
      out[2 * k] = (uint32_t)acc[k];
      out[2 * k + 1] = (uint32_t)(acc[k] >> 32);
    }
    __hip_atomic_store(out + 6, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

}  // namespace oo_rx

namespace {
int grid_for(uint32_t items) {
  const uint32_t g = (items + 255u) / 256u;
  return (int)(g < 1024u ? (g ? g : 1u) : 1024u);
}
}  // namespace

// kx_mode 1 (at most TABLE_THREADS ops): the incremental index update after
// the ops; kx_req is host memory the kernel sets to ask for a full rebuild.
extern "C" int oo_table_launch_ops(const oo_rx::DevTables* T, const oo_rx::TableOp* d_ops,
                                   const uint32_t* d_lev_end, uint32_t nlev, uint32_t gen,
                                   uint32_t kx_mode, uint32_t* kx_req, hipStream_t s) {
  hipLaunchKernelGGL(oo_rx::table_ops, dim3(1), dim3(oo_rx::TABLE_THREADS), 0, s, *T, d_ops,
                     d_lev_end, nlev, gen, kx_mode, kx_req);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" uint32_t oo_table_threads(void) { return oo_rx::TABLE_THREADS; }

extern "C" int oo_table_launch_refresh(const oo_rx::DevTables* T, uint32_t gen, hipStream_t s) {
  hipLaunchKernelGGL(oo_rx::table_refresh, dim3(grid_for(T->ip4_mask + T->ip6_mask + 2u)),
                     dim3(256), 0, s, *T, gen);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int oo_table_launch_init(const oo_rx::DevTables* T, hipStream_t s) {
  hipLaunchKernelGGL(oo_rx::table_init,
                     dim3(grid_for(T->ip4_mask + T->ip6_mask + 2u + T->max_socks)), dim3(256), 0,
                     s, *T);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Bytes of the two index arrays (oo_rx_device.h).
extern "C" uint64_t oo_table_kx_bytes4(uint32_t nb4) {
  return 2ull * (nb4 + oo_rx::KX_PAD4) * 32u;
}
extern "C" uint64_t oo_table_kx_bytes6(uint32_t ne6) {
  return (uint64_t)(ne6 + oo_rx::KX_PAD6) * 64u;
}

// The key index from the current tables, on s after the change that made
// them: cleared, marked usable, rebuilt (each check that fails marks it off).
extern "C" int oo_table_launch_kx(const oo_rx::DevTables* T, hipStream_t s) {
  if (T->kx4 == nullptr) return 0;
  if (hipMemsetAsync(T->kx4, 0, oo_table_kx_bytes4(T->kx_nb4), s) != hipSuccess ||
      hipMemsetAsync(T->kx6, 0, oo_table_kx_bytes6(T->kx_ne6), s) != hipSuccess ||
      hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(T->kx_ok), 1, 1, s) != hipSuccess)
    return -1;
  hipLaunchKernelGGL(oo_rx::table_kx, dim3(grid_for(T->ip4_mask + T->ip6_mask + 2u)), dim3(256), 0, s,
                     *T);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int oo_table_launch_occ(const oo_rx::DevTables* T, hipStream_t s) {
  hipLaunchKernelGGL(oo_rx::table_occ, dim3(grid_for((T->ip4_mask + T->ip6_mask + 2u) / 32u + 2u)),
                     dim3(256), 0, s, *T);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// The frame-length sample of a batch into host memory `out` (7 words: count,
// sum, sum of squares as u64 pairs, then seq), on s after the batch.
extern "C" int oo_launch_len_sample(const void* desc, uint32_t n, uint32_t ring_mask, uint32_t cons,
                                    uint32_t* out, uint32_t seq, hipStream_t s) {
  hipLaunchKernelGGL(oo_rx::len_sample, dim3(1), dim3(256), 0, s,
                     static_cast<const uint8_t*>(desc), n, ring_mask, cons, out, seq);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
