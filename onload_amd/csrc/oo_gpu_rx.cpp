// SPDX-License-Identifier: BSD-2-Clause
//
// oo_gpu_rx.cpp -- host side of the C ABI declared in include/oo_gpu_rx.h:
// context lifetime, the filter-table mirror (insert/remove with the
// reference's slot placement, route counts and tombstones), the op queue
// that carries every table change to the device copy (applied there by
// oo_table_kernel.hip on the batch stream), cross-stream ordering, the
// device-resident / AF_XDP / TX entry points, and the asynchronous
// host-memory path (pinned staging, two streams, double-buffered).
//
// Table semantics restated from (file:line in /root/reference):
//   ci_ip4_netif_filter_insert        src/lib/transport/ip/netif_table.c:323-406
//   ci_ip4_netif_filter_remove        netif_table.c:409-495
//   ci_ip4_netif_filter_lookup        netif_table.c:86-143
//   ci_ip6_netif_filter_insert        src/lib/transport/ip/netif_table_ip6.c:192-262
//   ci_ip6_netif_filter_remove        netif_table_ip6.c:264-345
//   ci_ip6_netif_filter_lookup        netif_table_ip6.c:13-66
//   ci_netif_filter_init / _ip6_init  netif_table.c:592-611, netif_table_ip6.c:349-365
//   __onload_hash1/2/3, addr_xor      src/include/onload/hash.h:31-173
#include <hip/hip_runtime_api.h>

#include <errno.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <map>
#include <mutex>
#include <new>
#include <unordered_map>
#include <unordered_set>
#include <string>
#include <vector>

#include "oo_rx_device.h"

extern "C" int oo_rx_launch(const oo_rx::KParams* P, int grid, hipStream_t stream);
extern "C" int oo_tx_launch(const oo_rx::KParams* P, int grid, hipStream_t stream);
extern "C" int oo_rx_blocks_per_cu(void);
extern "C" int oo_rx_launch_short(const oo_rx::KParams* P, int grid, hipStream_t stream);
extern "C" int oo_rx_blocks_per_cu_short(void);
extern "C" int oo_rx_waves_per_block(void);
extern "C" int oo_rx_launch_poll(const oo_rx::PollArgs* A, int grid, hipStream_t stream);
extern "C" int oo_rx_blocks_per_cu_poll(void);
extern "C" int oo_rx_win_blocks_per_cu(void);
extern "C" int oo_rx_body_blocks_per_cu(void);
extern "C" int oo_rx_win_waves_per_block(void);
extern "C" int oo_rx_body_waves_per_block(void);
extern "C" int oo_rx_launch_win(const oo_rx::KParams* P, int grid, hipStream_t stream);
extern "C" int oo_rx_launch_body(const oo_rx::KParams* P, int grid, hipStream_t stream);
extern "C" int oo_rx_body_blocks_per_cu_gseq(void);
extern "C" int oo_rx_launch_body_gseq(const oo_rx::KParams* P, int grid, hipStream_t stream);
extern "C" int oo_table_launch_ops(const oo_rx::DevTables* T, const oo_rx::TableOp* d_ops,
                                   const uint32_t* d_lev_end, uint32_t nlev, uint32_t gen,
                                   uint32_t kx_mode, uint32_t* kx_req, hipStream_t s);
extern "C" uint32_t oo_table_threads(void);
extern "C" int oo_launch_len_sample(const void* desc, uint32_t n, uint32_t ring_mask, uint32_t cons,
                                    uint32_t* out, uint32_t seq, hipStream_t s);
extern "C" int oo_table_launch_refresh(const oo_rx::DevTables* T, uint32_t gen, hipStream_t s);
extern "C" int oo_table_launch_init(const oo_rx::DevTables* T, hipStream_t s);
extern "C" int oo_table_launch_occ(const oo_rx::DevTables* T, hipStream_t s);
extern "C" int oo_table_launch_kx(const oo_rx::DevTables* T, hipStream_t s);
extern "C" uint64_t oo_table_kx_bytes4(uint32_t nb4);
extern "C" uint64_t oo_table_kx_bytes6(uint32_t ne6);

namespace {

using oo_rx::DevTables;
using oo_rx::hash2;
using oo_rx::hash3;
using oo_rx::ID6_EMPTY;
using oo_rx::ID6_TOMBSTONE;
using oo_rx::ID_MASK;
using oo_rx::KParams;
using oo_rx::occupied;
using oo_rx::Slot4;
using oo_rx::Slot6;
using oo_rx::ST_EMPTY;
using oo_rx::ST_MASK;
using oo_rx::ST_PREFERRED;
using oo_rx::ST_REHASHED;
using oo_rx::ST_TOMBSTONE;
using oo_rx::TableOp;


inline uint32_t ld32(const void* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}
inline uint32_t addr_xor(const void* a16) {
  const uint8_t* a = static_cast<const uint8_t*>(a16);
  return ld32(a) ^ ld32(a + 4) ^ ld32(a + 8) ^ ld32(a + 12);
}

// ci_netif_filter_table_entry_fast {id|state, laddr} and _ext
// {route_count, lport} (ip_shared_types.h:533-563).
struct Entry4 {
  uint32_t id_state, laddr;
};
struct Ext4 {
  int32_t route_count;
  uint16_t lport, pad;
};
// ci_ip6_netif_filter_table_entry {id, route_count, laddr[16]}
// (ip_shared_types.h:579-583).
struct Entry6 {
  int32_t id;
  int32_t route_count;
  uint32_t laddr[4];
};
static_assert(sizeof(Entry4) == 8 && sizeof(Ext4) == 8 && sizeof(Entry6) == 24,
              "entry layouts");

#ifndef OO_KX_LOG2_MAX
#define OO_KX_LOG2_MAX 17  // key index: buckets per IPv4 region / IPv6 entries at most, log2
#endif
#ifndef OO_KX_V4_MUL
#define OO_KX_V4_MUL 1  // IPv4 buckets per protocol region per table slot
#endif
#ifndef OO_KX_V6_MUL
#define OO_KX_V6_MUL 8  // IPv6 index entries per table slot (8: config 5 -0.3 % against 4, profiles/r06/ab_kx_sizes_c4_c5.log)
#endif
constexpr uint32_t OPS_CHUNK = 8192;  // table ops per device flush chunk (512 KiB)
constexpr uint32_t SMALL_N = 2048;    // launch(): batches up to this many packets take 8-packet tiles
// The poll instance (auto) up to OO_POLL_MAX packets -- a poll's batch:
// tools/poll_bench, DESIGN.md §5e -- writing a submit_mapped batch's done
// word itself up to OO_POLL_DONE_MAX (0: the instance never runs).
#ifndef OO_POLL_MAX
#define OO_POLL_MAX 256
#endif
#define OO_POLL_INSTANCE (OO_POLL_MAX > 0)
#ifndef OO_POLL_DONE_MAX
#define OO_POLL_DONE_MAX 2048
#endif
constexpr int NTRACK = 8;             // streams tracked at once (LRU)
constexpr int NSLOT = 2;              // host-path staging slots (double buffering)
// Host words the device writes and the host polls (done words, the length
// sample, the key index's rebuild request): fine-grained, so the GPU does not
// hold them in its L2 -- they are freed with the context.
constexpr unsigned kGpuWritten = hipHostMallocMapped | hipHostMallocCoherent;
// Tile-claim counter sets: two per tracked stream (its launches alternate
// between them), oo_rx::CLAIM_LINES lines of 128 B each (both kernels' group
// counters and the body flag).
constexpr uint32_t CLAIM_SETS = 2 * NTRACK;
using oo_rx::CLAIM_GROUPS;

// One stream the context launches on.  Nothing is recorded per launch: a
// table change (flush_ops) records `ev` on every other stream that launched
// since the last change and makes its own stream wait for it, which orders
// the change after every batch already enqueued there.  The entry's index
// also picks the stream's two tile-claim counter sets: launches on one stream
// run in order and alternate between them, each zeroing the other as it
// starts; an entry handed to another stream makes that stream wait for the
// old one first (track_of).
struct Tracked {
  hipStream_t s = nullptr;
  hipEvent_t ev = nullptr;
  bool used = false;      // assigned to s
  bool live = false;      // launched on s since a table change last ordered itself after s
  bool gone = false;      // oo_gpu_rx_stream_done: ev already covers all of s's work
  uint32_t parity = 0;    // claim set of the next launch (of the entry's two)
  uint32_t tables_seen = 0;  // table generation this stream has waited for
  uint64_t lru = 0;
  uint64_t* pend = nullptr;  // the split transform's pending words (launch_split)
  uint64_t pend_n = 0;
};

// One op-flush staging buffer: pinned host ops -> device ops, reused once
// the kernel that read it has finished (ev).
struct OpStage {
  TableOp* h = nullptr;
  TableOp* d = nullptr;
  hipEvent_t ev = nullptr;
  bool pending = false;
};

// One host-path staging slot (oo_gpu_rx_submit / _wait).
struct HostSlot {
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  uint8_t* d_frames = nullptr;
  oo_gpu_pkt_desc* d_desc = nullptr;
  oo_gpu_rx_result* d_out = nullptr;
  uint32_t* d_ctr = nullptr;
  uint8_t* h_frames = nullptr;  // pinned
  oo_gpu_pkt_desc* h_desc = nullptr;
  oo_gpu_rx_result* h_out = nullptr;
  uint32_t* h_ctr = nullptr;
  uint32_t* h_done = nullptr;  // pinned: the slot's last completed ticket (low 32 bits),
  uint32_t* d_done = nullptr;  //   written by the stream after the batch (complete_slot spins on it)
  bool busy = false;
  uint64_t ticket = 0;
  uint32_t n = 0;
  oo_gpu_rx_result* out = nullptr;  // caller's buffer
  oo_gpu_rx_counters* delta = nullptr;
  bool copy_out = false;  // out is not registered: copy from h_out at wait
};

struct HostReg {
  uintptr_t lo, hi;
  void* dev;
};

// Every range registered by any context of the process, by first byte: a
// registration is whole pages that no other registration shares
// (oo_gpu_rx_host_register; DESIGN.md §5 round 6, the registration faults).
std::mutex g_reg_mu;
std::map<uintptr_t, uintptr_t> g_reg_pages;  // lo -> hi

bool reg_overlaps(uintptr_t lo, uintptr_t hi) {
  auto it = g_reg_pages.lower_bound(lo);
  if (it != g_reg_pages.end() && it->first < hi) return true;
  return it != g_reg_pages.begin() && std::prev(it)->second > lo;
}

}  // namespace

struct oo_gpu_rx_ctx {
  int device = 0;
  uint32_t ip4_mask = 0, ip6_mask = 0, max_socks = 0;
  uint8_t hwport[OO_GPU_RX_MAX_INTF];
  // host mirror (authoritative for the calls that return at once)
  std::vector<Entry4> ip4;
  std::vector<Ext4> ip4_ext;
  std::vector<Entry6> ip6;
  std::vector<oo_gpu_rx_sock> socks;
  // device copy and the ops that have not reached it yet
  DevTables T = {};
  std::vector<TableOp> ops;
  bool ops_sock = false;  // ops holds an OP_SOCK (a refresh pass follows)
  // Parallel application (table_ops): each pending op's level -- one more
  // than the highest level of an earlier pending op that touched any slot
  // it touches (the probe walk the mirror just did) -- so ops of one level
  // touch disjoint slots and commute; levels run in order.  Socket ops are
  // level 0 (the refresh pass rewrites every slot of a changed socket after
  // all of them), and a later op on the same socket supersedes an earlier
  // one.
  std::vector<uint32_t> op_level;
  std::unordered_map<uint64_t, uint32_t> slot_level;  // (af << 32 | slot) -> first free level
  std::unordered_map<int32_t, size_t> sock_op_at;     // socket id -> its pending OP_SOCK
  std::vector<uint32_t> touched;                      // the last mirror op's probe walk
  uint32_t gen = 1;       // flush generation (sockgen marks)
  uint32_t tables_gen = 0;  // flushes done; streams wait for it via tables_ev
  uint64_t changes = 0;     // table / socket changes made (oo_gpu_rx_table_gen)
  uint32_t last_path = 0;   // the last RX batch's kernels (oo_gpu_rx_last_path)
  hipEvent_t tables_ev = nullptr;
  hipStream_t tables_stream = nullptr;
  OpStage stage[2];
  int stage_next = 0;
  // Key-index maintenance (oo_table_kernel.hip): a flush of at most
  // oo_table_threads() filter ops updates the ops' own keys in the ops
  // kernel; anything else rebuilds the index.  kx_full: the pending ops need
  // the rebuild (a socket change, or an op whose tuple is not its socket's);
  // h_kx_req: host memory a kernel sets when the index needs one (it is off,
  // or overflowed).
  bool kx_full = false;
  uint32_t* h_kx_req = nullptr;
  uint32_t* d_kx_req = nullptr;
  uint64_t n_flush = 0, n_kx_full = 0, n_kx_inc = 0;
  uint64_t n_kx_inc_run = 0;  // incremental updates since the last rebuild
  Tracked track[NTRACK];
  uint64_t lru = 0;
  uint8_t* d_zero = nullptr;   // oo_rx::ZERO_LINES x 16 B of zeros, the sink, the hwport table
  uint32_t* d_claim = nullptr; // CLAIM_SETS x CLAIM_LINES words, 128 B apart
  bool failed = false;         // a table flush failed part-way: the device copy is unknown
  bool dyn = true;             // dynamic tile claims (OO_RX_STATIC=1: static)
  uint32_t tail_tile = 32;     // packets per tile at the batch's end (dynamic)
  uint32_t tail_per_wave = 1;  // such tiles per wave
  uint32_t ngroups_max = 0;    // claim groups at most (0: chosen per launch)
  uint32_t gshift = ~0u;       // claim group of a wave: (gwave >> gshift) mod groups (~0u: per launch)
  uint32_t grid = 1024;        // resident blocks of rx_kernel
  uint32_t grid_short = 0;     // resident blocks of the short-frame rx_kernel (0: unused)
  uint32_t grid_poll = 0;      // resident blocks of the poll instance's rx_kernel (0: unused)
  // A submit_mapped batch's completion, handed to launch(): the slot's done
  // word and value; launch() sets done_by_kernel when the poll instance
  // writes it.
  uint32_t* poll_done = nullptr;
  uint32_t poll_done_val = 0;
  bool done_by_kernel = false;
  std::vector<void*> retired;  // replaced pending-word buffers (freed at close)
  uint32_t ncu = 0, bpc[6] = {0, 0, 0, 0, 0, 0};  // CUs; resident blocks per CU of the six kernels
  uint32_t grid_win = 0;       // resident blocks of win_kernel (split transform)
  uint32_t grid_body = 0;      // resident blocks of body_kernel
  uint32_t grid_body_gseq = 0; // ... of its per-group-sequence instance
  uint32_t body_engine = 0;    // oo_gpu_rx_tuning::body_engine
  bool kx = true;              // lookups through the key index (oo_gpu_rx_tuning::walks)
  uint32_t body_tail = 16;     // packets per body_kernel unit at the batch's end
  uint32_t kmode = 0;          // rx kernel: 0 by frame size, 1 always the 4-slot, 2 always the 2-slot
  uint32_t len_hint = 0;       // mean frame length of the batches to come (0: from buffer bytes)
  // The frame-length profile of the last batch sampled without a hint
  // (launch(): mixed sizes take the split transform).  A batch whose
  // descriptors (address, count, ring position) differ from the last sampled
  // one gets a sample after it (oo_table_kernel.hip len_sample, into host
  // memory); launches with the same descriptors use it once its event has
  // completed -- nothing waits for it.
  uint32_t* h_len = nullptr;
  uint32_t* d_len = nullptr;
  hipEvent_t len_ev = nullptr;
  const void* len_desc = nullptr;
  uint32_t len_n = 0, len_cons = 0, len_seq = 0;
  uint32_t len_uses = 0;       // launches on the sampled key since its sample
  bool len_pending = false;
  bool host_batch = false;     // launch() runs oo_gpu_rx_submit's batch: no sample
  int len_mixed = -1;          // the sampled batch: 1 mixed sizes, 0 not, -1 not known yet
  uint32_t tstep = 8;          // tile size step (KParams::tstep)
  uint64_t* stamps = nullptr;  // diagnostic phase stamps (OO_RX_STAMPS builds)
  // host path
  uint64_t stage_bytes = 0;
  uint32_t stage_pkts = 0;
  HostSlot slot[NSLOT];
  uint64_t next_ticket = 1;
  std::vector<HostReg> regs;
  hipStream_t stream = nullptr;  // the context's own stream (setup work)
  uint8_t* h_image_hdr = nullptr;  // pinned 64-B table image header
};

// A slot's done word seen by spinning (below).
static bool spin_done(const HostSlot& s);

namespace {

bool has_dev(const oo_gpu_rx_ctx* c) { return c->device >= 0; }

// Queues op for the device.  A table op's level comes from the slots its
// mirror walk touched (c->touched); a socket op supersedes the socket's
// pending one.
void push_op(oo_gpu_rx_ctx* c, const TableOp& op) {
  if (!has_dev(c)) return;
  uint32_t level = 0;
  if (op.kind == oo_rx::OP_SOCK) {
    c->ops_sock = true;
    auto it = c->sock_op_at.find(op.sock);
    if (it != c->sock_op_at.end()) c->ops[it->second].kind = 0;  // superseded: skipped
    c->sock_op_at[op.sock] = c->ops.size();
  } else {
    // The index keys an op's entry by its socket's fields (the slot record's);
    // an op whose tuple differs cannot be updated incrementally.
    const oo_gpu_rx_sock& k = c->socks[op.sock];
    const bool same = op.af == 4 ? op.u.t.ra[0] == k.raddr_be32 && op.rport == k.rport_be16 &&
                                       op.proto == k.protocol
                                 : memcmp(op.u.t.ra, k.raddr6, 16) == 0 && op.rport == k.rport_be16 &&
                                       op.lport == k.lport_be16 && op.proto == k.protocol;
    if (!same) c->kx_full = true;
    const uint64_t af = (uint64_t)op.af << 32;
    for (uint32_t slot : c->touched) {
      auto it = c->slot_level.find(af | slot);
      if (it != c->slot_level.end()) level = std::max(level, it->second);
    }
    for (uint32_t slot : c->touched) c->slot_level[af | slot] = level + 1;
  }
  c->ops.push_back(op);
  c->op_level.push_back(level);
}

void clear_ops(oo_gpu_rx_ctx* c) {
  c->kx_full = false;
  c->ops.clear();
  c->op_level.clear();
  c->slot_level.clear();
  c->sock_op_at.clear();
  c->ops_sock = false;
}

TableOp tuple_op(uint8_t kind, int af, const void* la, uint16_t lp, const void* ra, uint16_t rp,
                 uint8_t proto, int32_t id) {
  TableOp op;
  memset(&op, 0, sizeof(op));
  op.kind = kind;
  op.af = (uint8_t)af;
  op.proto = proto;
  op.lport = lp;
  op.rport = rp;
  op.sock = id;
  const size_t n = af == 4 ? 4 : 16;
  memcpy(op.u.t.la, la, n);
  if (ra) memcpy(op.u.t.ra, ra, n);
  return op;
}

// ---- IPv4 mirror: netif_table.c:323-495.
// Each mirror op leaves the slots its walk touched in c->touched.
int ip4_insert(oo_gpu_rx_ctx* c, int32_t id, uint32_t la, uint32_t lp, uint32_t ra,
               uint32_t rp, uint32_t proto) {
  uint32_t h1 = hash3(la, lp, ra, rp, proto) & c->ip4_mask;
  const uint32_t h2 = hash2(la, lp, ra, rp, proto);
  const uint32_t first = h1;
  c->touched.clear();
  while (occupied(c->ip4[h1].id_state)) {
    c->touched.push_back(h1);
    ++c->ip4_ext[h1].route_count;
    h1 = (h1 + h2) & c->ip4_mask;
    if (h1 == first) return -ENOBUFS;  // route counts stay raised (:349-376)
  }
  c->touched.push_back(h1);
  c->ip4[h1].id_state = (h1 == first ? ST_PREFERRED : ST_REHASHED) | ((uint32_t)id & ID_MASK);
  c->ip4[h1].laddr = la;
  c->ip4_ext[h1].lport = (uint16_t)lp;
  return 0;
}

void ip4_remove(oo_gpu_rx_ctx* c, int32_t id, uint32_t la, uint32_t lp, uint32_t ra,
                uint32_t rp, uint32_t proto) {
  const uint32_t h1 = hash3(la, lp, ra, rp, proto) & c->ip4_mask;
  const uint32_t h2 = hash2(la, lp, ra, rp, proto);
  uint32_t i = h1;
  int hops = 0;
  c->touched.clear();
  for (;;) {
    c->touched.push_back(i);
    const uint32_t st = c->ip4[i].id_state;
    if (occupied(st) && (st & ID_MASK) == ((uint32_t)id & ID_MASK)) {
      if (la == c->ip4[i].laddr) break;
    } else if ((st & ST_MASK) == ST_EMPTY) {
      return;  // multiple removes are allowed (:476-481)
    }
    i = (i + h2) & c->ip4_mask;
    ++hops;
    if (i == h1) return;
  }
  i = h1;
  for (int k = 0; k < hops; ++k) {
    if (--c->ip4_ext[i].route_count == 0 && (c->ip4[i].id_state & ST_MASK) == ST_TOMBSTONE)
      c->ip4[i].id_state = (c->ip4[i].id_state & ID_MASK) | ST_EMPTY;
    i = (i + h2) & c->ip4_mask;
  }
  c->ip4[i].id_state =
      (c->ip4[i].id_state & ID_MASK) | (c->ip4_ext[i].route_count == 0 ? ST_EMPTY : ST_TOMBSTONE);
}

int ip4_lookup(const oo_gpu_rx_ctx* c, uint32_t la, uint32_t lp, uint32_t ra, uint32_t rp,
               uint32_t proto) {
  uint32_t h1 = hash3(la, lp, ra, rp, proto) & c->ip4_mask;
  const uint32_t first = h1;
  uint32_t h2 = 0;
  for (;;) {
    const uint32_t st = c->ip4[h1].id_state;
    if (occupied(st)) {
      const oo_gpu_rx_sock& s = c->socks[st & ID_MASK];
      if (la == c->ip4[h1].laddr && lp == c->ip4_ext[h1].lport && ra == s.raddr_be32 &&
          rp == s.rport_be16 && proto == s.protocol)
        return (int)h1;
    }
    if ((st & ST_MASK) == ST_EMPTY) break;
    if (h1 == first) h2 = hash2(la, lp, ra, rp, proto);
    h1 = (h1 + h2) & c->ip4_mask;
    if (h1 == first) return -ELOOP;
  }
  return -ENOENT;
}

// ---- IPv6 mirror: netif_table_ip6.c:13-345.
int ip6_insert(oo_gpu_rx_ctx* c, int32_t id, const uint8_t* la, uint32_t lp,
               const uint8_t* ra, uint32_t rp, uint32_t proto) {
  const uint32_t lx = addr_xor(la), rx = addr_xor(ra);
  uint32_t h1 = hash3(lx, lp, rx, rp, proto) & c->ip6_mask;
  const uint32_t h2 = hash2(lx, lp, rx, rp, proto);
  const uint32_t first = h1;
  c->touched.clear();
  while (c->ip6[h1].id >= 0) {
    c->touched.push_back(h1);
    ++c->ip6[h1].route_count;
    h1 = (h1 + h2) & c->ip6_mask;
    if (h1 == first) return -ENOBUFS;
  }
  c->touched.push_back(h1);
  c->ip6[h1].id = id;
  memcpy(c->ip6[h1].laddr, la, 16);
  return 0;
}

void ip6_remove(oo_gpu_rx_ctx* c, int32_t id, const uint8_t* la, uint32_t lp,
                const uint8_t* ra, uint32_t rp, uint32_t proto) {
  const uint32_t lx = addr_xor(la), rx = addr_xor(ra);
  const uint32_t h1 = hash3(lx, lp, rx, rp, proto) & c->ip6_mask;
  const uint32_t h2 = hash2(lx, lp, rx, rp, proto);
  uint32_t i = h1;
  int hops = 0;
  c->touched.clear();
  for (;;) {
    c->touched.push_back(i);
    const Entry6& e = c->ip6[i];
    if (e.id == id) {
      if (memcmp(la, e.laddr, 16) == 0) break;
    } else if (e.id == ID6_EMPTY) {
      return;
    }
    i = (i + h2) & c->ip6_mask;
    ++hops;
    if (i == h1) return;
  }
  i = h1;
  for (int k = 0; k < hops; ++k) {
    Entry6& e = c->ip6[i];
    if (--e.route_count == 0 && e.id == ID6_TOMBSTONE) e.id = ID6_EMPTY;
    i = (i + h2) & c->ip6_mask;
  }
  c->ip6[i].id = c->ip6[i].route_count == 0 ? ID6_EMPTY : ID6_TOMBSTONE;
}

int ip6_lookup(const oo_gpu_rx_ctx* c, const uint8_t* la, uint32_t lp, const uint8_t* ra,
               uint32_t rp, uint32_t proto) {
  const uint32_t lx = addr_xor(la), rx = addr_xor(ra);
  uint32_t h1 = hash3(lx, lp, rx, rp, proto) & c->ip6_mask;
  const uint32_t first = h1;
  uint32_t h2 = 0;
  for (;;) {
    const int32_t id = c->ip6[h1].id;
    if (id >= 0) {
      const oo_gpu_rx_sock& s = c->socks[id];
      if (lp == s.lport_be16 && rp == s.rport_be16 && proto == s.protocol &&
          memcmp(la, c->ip6[h1].laddr, 16) == 0 && memcmp(ra, s.raddr6, 16) == 0)
        return (int)h1;
    }
    if (id == ID6_EMPTY) break;
    if (h1 == first) h2 = hash2(lx, lp, rx, rp, proto);
    h1 = (h1 + h2) & c->ip6_mask;
    if (h1 == first) return -ELOOP;
  }
  return -ENOENT;
}

const uint8_t kZero16[16] = {0};

// ---- Table image (oo_gpu_rx_table_export / _import): a 64-B header, then
// the slot records as the device holds them (Slot4 + route counts, Slot6)
// and the socket records.
constexpr uint32_t IMAGE_MAGIC = 0x42544f4fu;  // "OOTB"
constexpr uint32_t IMAGE_VERSION = 1;
struct ImageHdr {
  uint32_t magic, version;
  uint32_t ip4_log2, ip6_log2, max_socks, rsvd0;
  uint64_t off_slot4, off_rc4, off_slot6, off_socks, total;

};
static_assert(sizeof(ImageHdr) == 64, "image header");

int log2u(uint32_t v) { return 31 - __builtin_clz(v); }

ImageHdr image_hdr(const oo_gpu_rx_ctx* c) {
  ImageHdr h;
  memset(&h, 0, sizeof(h));
  const uint64_t n4 = c->ip4_mask + 1ull, n6 = c->ip6_mask + 1ull;
  h.magic = IMAGE_MAGIC;
  h.version = IMAGE_VERSION;
  h.ip4_log2 = (uint32_t)log2u(c->ip4_mask + 1u);
  h.ip6_log2 = (uint32_t)log2u(c->ip6_mask + 1u);
  h.max_socks = c->max_socks;
  h.off_slot4 = sizeof(ImageHdr);
  h.off_rc4 = h.off_slot4 + n4 * sizeof(Slot4);
  h.off_slot6 = h.off_rc4 + n4 * sizeof(int32_t);
  h.off_socks = h.off_slot6 + n6 * sizeof(Slot6);
  h.total = h.off_socks + (uint64_t)c->max_socks * sizeof(oo_gpu_rx_sock);
  return h;
}

// The device record of a slot as the mirror defines it: entry fields, and
// the fields of the socket the id names while the slot is not EMPTY (IPv4)
// or occupied (IPv6); zero otherwise (oo_table_kernel.hip keeps the same).
Slot4 slot4_of(const oo_gpu_rx_ctx* c, uint32_t i) {
  Slot4 r;
  memset(&r, 0, sizeof(r));
  r.id_state = c->ip4[i].id_state;
  r.laddr = c->ip4[i].laddr;
  r.lport = c->ip4_ext[i].lport;
  const uint32_t id = r.id_state & ID_MASK;
  if ((r.id_state & ST_MASK) != ST_EMPTY && id < c->max_socks) {
    const oo_gpu_rx_sock& k = c->socks[id];
    r.raddr = k.raddr_be32;
    r.rport = k.rport_be16;
    r.proto = k.protocol;
    r.sflags = k.flags;
    r.b2d_vlan = k.bind2dev_vlan;
    r.hwports = k.bind2dev_hwports;
  }
  return r;
}

Slot6 slot6_of(const oo_gpu_rx_ctx* c, uint32_t i) {
  Slot6 r;
  memset(&r, 0, sizeof(r));
  const Entry6& e = c->ip6[i];
  r.id = e.id;
  r.route_count = e.route_count;
  memcpy(r.laddr, e.laddr, 16);
  if (e.id >= 0 && (uint32_t)e.id < c->max_socks) {
    const oo_gpu_rx_sock& k = c->socks[e.id];
    memcpy(r.raddr, k.raddr6, 16);
    r.lport = k.lport_be16;
    r.rport = k.rport_be16;
    r.proto = k.protocol;
    r.sflags = k.flags;
    r.b2d_vlan = k.bind2dev_vlan;
    r.hwports = k.bind2dev_hwports;
  }
  return r;
}

void image_from_mirror(const oo_gpu_rx_ctx* c, uint8_t* dst) {
  const ImageHdr h = image_hdr(c);
  memcpy(dst, &h, sizeof(h));
  Slot4* s4 = reinterpret_cast<Slot4*>(dst + h.off_slot4);
  int32_t* rc4 = reinterpret_cast<int32_t*>(dst + h.off_rc4);
  Slot6* s6 = reinterpret_cast<Slot6*>(dst + h.off_slot6);
  for (uint32_t i = 0; i <= c->ip4_mask; ++i) {
    s4[i] = slot4_of(c, i);
    rc4[i] = c->ip4_ext[i].route_count;
  }
  for (uint32_t i = 0; i <= c->ip6_mask; ++i) s6[i] = slot6_of(c, i);
  memcpy(dst + h.off_socks, c->socks.data(), sizeof(oo_gpu_rx_sock) * c->max_socks);
}

void mirror_from_image(oo_gpu_rx_ctx* c, const uint8_t* src) {
  const ImageHdr h = image_hdr(c);
  const Slot4* s4 = reinterpret_cast<const Slot4*>(src + h.off_slot4);
  const int32_t* rc4 = reinterpret_cast<const int32_t*>(src + h.off_rc4);
  const Slot6* s6 = reinterpret_cast<const Slot6*>(src + h.off_slot6);
  for (uint32_t i = 0; i <= c->ip4_mask; ++i) {
    c->ip4[i].id_state = s4[i].id_state;
    c->ip4[i].laddr = s4[i].laddr;
    c->ip4_ext[i].lport = s4[i].lport;
    c->ip4_ext[i].route_count = rc4[i];
  }
  for (uint32_t i = 0; i <= c->ip6_mask; ++i) {
    c->ip6[i].id = s6[i].id;
    c->ip6[i].route_count = s6[i].route_count;
    memcpy(c->ip6[i].laddr, s6[i].laddr, 16);
  }
  memcpy(c->socks.data(), src + h.off_socks, sizeof(oo_gpu_rx_sock) * c->max_socks);
}

// ---- Device lifetime.
void free_dev(oo_gpu_rx_ctx* c) {
  DevTables& T = c->T;
  for (void* p : {(void*)T.slot4, (void*)T.rc4, (void*)T.occ4, (void*)T.slot6, (void*)T.occ6,
                  (void*)T.socks, (void*)T.sockgen, (void*)c->d_zero, (void*)c->d_claim,
                  (void*)T.kx4, (void*)T.kx6, (void*)T.kx_ok})
    if (p) (void)hipFree(p);
  for (OpStage& st : c->stage) {
    if (st.h) (void)hipHostFree(st.h);
    if (st.d) (void)hipFree(st.d);
    if (st.ev) (void)hipEventDestroy(st.ev);
  }
  for (HostSlot& s : c->slot) {
    for (void* p : {(void*)s.d_frames, (void*)s.d_desc, (void*)s.d_out, (void*)s.d_ctr})
      if (p) (void)hipFree(p);
    for (void* p : {(void*)s.h_frames, (void*)s.h_desc, (void*)s.h_out, (void*)s.h_ctr, (void*)s.h_done})
      if (p) (void)hipHostFree(p);
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.stream) (void)hipStreamDestroy(s.stream);
  }
  for (Tracked& t : c->track) {
    if (t.ev) (void)hipEventDestroy(t.ev);
    if (t.pend) (void)hipFree(t.pend);
  }
  for (void* p : c->retired) (void)hipFree(p);
  if (c->tables_ev) (void)hipEventDestroy(c->tables_ev);
  if (c->h_image_hdr) (void)hipHostFree(c->h_image_hdr);
  if (c->h_kx_req) (void)hipHostFree(c->h_kx_req);
  if (c->h_len) (void)hipHostFree(c->h_len);
  if (c->len_ev) (void)hipEventDestroy(c->len_ev);
  if (c->stream) (void)hipStreamDestroy(c->stream);
}

// An event that completes once everything enqueued on t's stream so far
// has: recorded now (a stream given up with oo_gpu_rx_stream_done already
// has its final one).
hipEvent_t mark(Tracked& t) {
  if (!t.gone && hipEventRecord(t.ev, t.s) != hipSuccess) return nullptr;
  return t.ev;
}

// The tracked entry of stream s (the least recently used one reassigned).
// Reassigning an entry makes s wait for everything enqueued on its old
// stream: that frees the entry's claim counters for s, and s carries the
// old stream's table reads (live) into the next table change.  Returns
// nullptr on a HIP failure.
Tracked* track_of(oo_gpu_rx_ctx* c, hipStream_t s) {
  Tracked* victim = &c->track[0];
  for (Tracked& t : c->track) {
    if (t.used && !t.gone && t.s == s) {
      t.lru = ++c->lru;
      return &t;
    }
    if (!t.used) {
      victim = &t;
      break;
    }
    if (t.lru < victim->lru) victim = &t;
  }
  bool live = false;
  if (victim->ev == nullptr) {
    if (hipEventCreateWithFlags(&victim->ev, hipEventDisableTiming) != hipSuccess) return nullptr;
  } else if (victim->used) {
    hipEvent_t e = mark(*victim);
    if (e == nullptr || hipStreamWaitEvent(s, e, 0) != hipSuccess) return nullptr;
    live = victim->live;
  }
  victim->s = s;
  victim->used = true;
  victim->gone = false;
  victim->live = live;
  victim->tables_seen = 0;
  victim->lru = ++c->lru;
  return victim;
}

uint32_t track_index(const oo_gpu_rx_ctx* c, const Tracked* t) { return (uint32_t)(t - c->track); }

// Stream s follows every batch enqueued on another stream that may still
// read the tables (no batch sees a half-updated table).
int order_after_batches(oo_gpu_rx_ctx* c, hipStream_t s) {
  for (Tracked& t : c->track) {
    if (t.used && t.live && (t.gone || t.s != s)) {
      hipEvent_t e = mark(t);
      if (e == nullptr || hipStreamWaitEvent(s, e, 0) != hipSuccess) return -EIO;
      t.live = false;
    }
  }
  return 0;
}

// One op per distinct index key of an incremental flush recomputes it
// (TableOp::rsvd0 KX_OWN_*): the exact tuple, and for IPv6 the wildcard key
// (laddr, lport, protocol) of the ra_null stages.
void mark_kx_owners(TableOp* h, uint32_t n) {
  std::unordered_set<std::string> seen;
  for (uint32_t k = 0; k < n; ++k) {
    TableOp& op = h[k];
    if (op.kind != oo_rx::OP_INSERT && op.kind != oo_rx::OP_REMOVE) continue;
    std::string key(reinterpret_cast<const char*>(&op.u.t), sizeof(op.u.t));
    key.push_back((char)op.af);
    key.push_back((char)op.proto);
    key.append(reinterpret_cast<const char*>(&op.lport), 2);
    std::string wild = key;
    key.append(reinterpret_cast<const char*>(&op.rport), 2);
    if (seen.insert(key).second) op.rsvd0 |= oo_rx::KX_OWN_EXACT;
    if (op.af == 6) {
      memset(&wild[16], 0, 16);  // (raddr)
      wild.push_back('w');
      if (seen.insert(wild).second) op.rsvd0 |= oo_rx::KX_OWN_WILD;
    }
  }
}

// Pending table ops -> device, on stream s: first order s after the
// batches on other streams, then copy the ops through a pinned staging
// buffer and apply them (table_ops), then refresh the socket fields of the
// slots whose socket changed.  No host synchronisation unless a staging
// buffer is still in use by an earlier flush that has not run.  A failure
// after the first chunk has been enqueued leaves the device tables in an
// unknown state: the context then refuses every later call (-EIO) rather
// than apply the queued ops twice.
// With no ops queued it only rebuilds the key index (index_due): the
// index asked for it, or has had kKxIncMax incremental updates since its
// last rebuild (a key that lost its last match keeps a KX_DEAD entry, whose
// lookups walk: ADVICE r5).
constexpr uint64_t kKxIncMax = 256;
bool index_due(const oo_gpu_rx_ctx* c) {
  if (c->T.kx4 == nullptr || c->h_kx_req == nullptr) return false;
  return *reinterpret_cast<const volatile uint32_t*>(c->h_kx_req) != 0 || c->n_kx_inc_run >= kKxIncMax;
}

int flush_ops(oo_gpu_rx_ctx* c, hipStream_t s) {
  if (c->ops.empty() && !index_due(c)) return 0;
  if (order_after_batches(c, s) != 0) return -EIO;
  // The ops in level order (call order within a level), cut into chunks;
  // each chunk carries the end of every level it holds part of.
  const uint32_t total = (uint32_t)c->ops.size();
  std::vector<uint32_t> order(total);
  for (uint32_t i = 0; i < total; ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(),
                   [c](uint32_t a, uint32_t b) { return c->op_level[a] < c->op_level[b]; });
  // A small flush with filter ops only and the index not asking for a
  // rebuild updates the index for the ops' keys.
  const bool small = total <= oo_table_threads();
  const bool req = c->h_kx_req != nullptr && *reinterpret_cast<volatile uint32_t*>(c->h_kx_req) != 0;
  const bool inc = total > 0 && small && !c->kx_full && !c->ops_sock && !req &&
                   c->n_kx_inc_run < kKxIncMax && c->d_kx_req != nullptr && c->T.kx4 != nullptr;
  for (uint32_t at = 0; at < total; at += OPS_CHUNK) {
    const uint32_t n = std::min(OPS_CHUNK, total - at);
    OpStage& st = c->stage[c->stage_next];
    c->stage_next ^= 1;
    if (st.pending && hipEventSynchronize(st.ev) != hipSuccess) {
      c->failed = at > 0;
      return -EIO;
    }
    TableOp* h = st.h;
    uint32_t* lev_end = reinterpret_cast<uint32_t*>(h + OPS_CHUNK);
    uint32_t nlev = 0;
    for (uint32_t k = 0; k < n; ++k) {
      const uint32_t i = order[at + k];
      h[k] = c->ops[i];
      h[k].rsvd0 = 0;
      if (k > 0 && c->op_level[i] != c->op_level[order[at + k - 1]]) lev_end[nlev++] = k;
    }
    lev_end[nlev++] = n;
    if (inc) mark_kx_owners(h, n);
    // (Copied to device memory even when small: the kernel does not read
    // host memory in place -- DESIGN.md §5 round 5, the faults.)
    const TableOp* d_ops = st.d;
    const uint32_t* d_lev = reinterpret_cast<const uint32_t*>(st.d + OPS_CHUNK);
    const bool ok =
        hipMemcpyAsync(st.d, st.h, sizeof(TableOp) * n, hipMemcpyHostToDevice, s) == hipSuccess &&
        hipMemcpyAsync(st.d + OPS_CHUNK, lev_end, sizeof(uint32_t) * nlev, hipMemcpyHostToDevice, s) ==
            hipSuccess;
    if (!ok || oo_table_launch_ops(&c->T, d_ops, d_lev, nlev, c->gen, inc ? 1u : 0u, c->d_kx_req, s) != 0 ||
        hipEventRecord(st.ev, s) != hipSuccess) {
      c->failed = true;  // this chunk or an earlier one may have reached the device
      return -EIO;
    }
    st.pending = true;
  }
  if (!inc && c->h_kx_req != nullptr) *reinterpret_cast<volatile uint32_t*>(c->h_kx_req) = 0;
  if ((c->ops_sock && oo_table_launch_refresh(&c->T, c->gen, s) != 0) ||
      (!inc && oo_table_launch_kx(&c->T, s) != 0)) {
    c->failed = true;
    return -EIO;
  }
  if (total > 0) ++c->n_flush;
  ++(inc ? c->n_kx_inc : c->n_kx_full);
  c->n_kx_inc_run = inc ? c->n_kx_inc_run + 1 : 0;
  if (total > 0) {
    clear_ops(c);
    ++c->gen;
  }
  ++c->tables_gen;
  Tracked* t = track_of(c, s);
  if (t == nullptr || hipEventRecord(c->tables_ev, s) != hipSuccess) {
    c->failed = true;
    return -EIO;
  }
  c->tables_stream = s;
  t->tables_seen = c->tables_gen;
  return 0;
}

// Everything a launch on stream s must follow: pending table ops, or the
// last flush when it ran on another stream.  Returns s's tracked entry.
int prepare(oo_gpu_rx_ctx* c, hipStream_t s, Tracked** out = nullptr) {
  if (c->failed) return -EIO;
  if (!c->ops.empty() || index_due(c)) {
    const int rc = flush_ops(c, s);
    if (rc) return rc;
  }
  Tracked* t = track_of(c, s);
  if (t == nullptr) return -EIO;
  if (c->tables_gen != 0 && t->tables_seen != c->tables_gen) {
    if (c->tables_stream != s && hipStreamWaitEvent(s, c->tables_ev, 0) != hipSuccess)
      return -EIO;
    t->tables_seen = c->tables_gen;
  }
  if (out) *out = t;
  return 0;
}

// A launch (or copy) on s that reads the tables: the next table change
// orders itself after it.
void note_launch(Tracked* t) { t->live = true; }

bool in_reg(const oo_gpu_rx_ctx* c, const void* p, uint64_t bytes) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  for (const HostReg& r : c->regs)
    if (a >= r.lo && a <= r.hi && bytes <= r.hi - a) return true;
  return false;
}

int alloc_host_slots(oo_gpu_rx_ctx* c) {
  for (HostSlot& s : c->slot) {
    const uint64_t pk = c->stage_pkts;
    if (hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&s.done, hipEventDisableTiming) != hipSuccess ||
        hipMalloc(&s.d_frames, c->stage_bytes) != hipSuccess ||
        hipMalloc(&s.d_desc, sizeof(oo_gpu_pkt_desc) * pk) != hipSuccess ||
        hipMalloc(&s.d_out, sizeof(oo_gpu_rx_result) * pk) != hipSuccess ||
        hipMalloc(&s.d_ctr, sizeof(oo_gpu_rx_counters)) != hipSuccess ||
        hipHostMalloc(&s.h_frames, c->stage_bytes, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&s.h_desc, sizeof(oo_gpu_pkt_desc) * pk, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&s.h_out, sizeof(oo_gpu_rx_result) * pk, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&s.h_ctr, sizeof(oo_gpu_rx_counters), hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&s.h_done, 128, kGpuWritten) != hipSuccess ||
        hipHostGetDevicePointer(reinterpret_cast<void**>(&s.d_done), s.h_done, 0) != hipSuccess)
      return -ENOMEM;
    *s.h_done = 0;
  }
  return 0;
}

// The launch settings (oo_gpu_rx_set_tuning; nullptr: the defaults).
void apply_tuning(oo_gpu_rx_ctx* c, const oo_gpu_rx_tuning* t) {
  oo_gpu_rx_tuning d;
  memset(&d, 0, sizeof(d));
  d.gshift = -1;
  if (t == nullptr) t = &d;
  const uint32_t pct = t->grid_pct ? t->grid_pct : 100u;
  auto grid = [&](uint32_t bpc) {
    return bpc ? std::max<uint32_t>(1, bpc * c->ncu * pct / 100u) : 0u;
  };
  c->grid = std::max<uint32_t>(1, grid(c->bpc[0]));
  c->grid_short = grid(c->bpc[1]);
  c->grid_win = grid(c->bpc[2]);
  c->grid_body = grid(t->body_bpc ? std::min(t->body_bpc, c->bpc[3]) : c->bpc[3]);
  c->grid_body_gseq = grid(t->body_bpc ? std::min(t->body_bpc, c->bpc[4]) : c->bpc[4]);
  c->grid_poll = OO_POLL_INSTANCE ? grid(c->bpc[5]) : 0u;
  c->body_engine = t->body_engine;
  c->kx = t->walks == 0;
  c->kmode = t->path;
  c->tstep = t->tstep == 1 ? 1 : 8;
  c->dyn = t->static_tiles == 0;
  c->tail_tile = std::min<uint32_t>(64, std::max<uint32_t>(8, (t->tail_tile ? t->tail_tile : 32) / 8 * 8));
  c->tail_per_wave = t->tail_per_wave ? t->tail_per_wave : 1;
  c->body_tail = std::min<uint32_t>(64, std::max<uint32_t>(8, (t->body_tail ? t->body_tail : 16) / 8 * 8));
  c->ngroups_max = std::min<uint32_t>(CLAIM_GROUPS, t->groups);  // 0: by frame size
  c->gshift = t->gshift < 0 ? ~0u : (uint32_t)t->gshift;         // ~0: by frame size
}

}  // namespace

extern "C" {

int oo_gpu_rx_abi_version(void) { return OO_GPU_RX_ABI_VERSION; }

int oo_gpu_rx_set_tuning(oo_gpu_rx_ctx* c, const oo_gpu_rx_tuning* t) {
  if (c == nullptr || (t != nullptr && (t->path > 4 || t->grid_pct > 100 || t->body_engine > 2 ||
                                  t->walks > 1))) return -EINVAL;
  apply_tuning(c, t);
  return 0;
}

int oo_gpu_rx_open(oo_gpu_rx_ctx** out, const oo_gpu_rx_cfg* cfg) {
  if (out == nullptr || cfg == nullptr) return -EINVAL;
  *out = nullptr;
  if (cfg->ip4_table_log2 < 16 || cfg->ip4_table_log2 > 24 || cfg->ip6_table_log2 < 1 ||
      cfg->ip6_table_log2 > 24 || cfg->max_socks == 0 || cfg->max_socks > (1u << 30) ||
      cfg->n_intf > OO_GPU_RX_MAX_INTF)
    return -EINVAL;
  // device < 0: a host-only context (the filter-table mirror without a GPU,
  // e.g. to build a table before a device is attached); batch calls fail
  // with -ENODEV.
  const bool host_only = cfg->device < 0;
  if (!host_only) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return -ENODEV;
    if (cfg->device >= ndev) return -ENODEV;
    if (hipSetDevice(cfg->device) != hipSuccess) return -ENODEV;
  }

  oo_gpu_rx_ctx* c = new (std::nothrow) oo_gpu_rx_ctx();
  if (c == nullptr) return -ENOMEM;
  c->device = cfg->device;
  c->ip4_mask = (1u << cfg->ip4_table_log2) - 1;
  c->ip6_mask = (1u << cfg->ip6_table_log2) - 1;
  c->max_socks = cfg->max_socks;
  memset(c->hwport, 0xff, sizeof(c->hwport));
  memcpy(c->hwport, cfg->intf_hwport, cfg->n_intf);
  try {
    c->ip4.assign(c->ip4_mask + 1, Entry4{ST_EMPTY, 0});
    c->ip4_ext.assign(c->ip4_mask + 1, Ext4{0, 0, 0});
    c->ip6.assign(c->ip6_mask + 1, Entry6{ID6_EMPTY, 0, {0, 0, 0, 0}});
    c->socks.assign(c->max_socks, oo_gpu_rx_sock{});
  } catch (...) {
    delete c;
    return -ENOMEM;
  }
  if (host_only) {
    *out = c;
    return 0;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, c->device) == hipSuccess && prop.multiProcessorCount > 0) {
    // Persistent grids: every resident block (occupancy query).
    c->ncu = (uint32_t)prop.multiProcessorCount;
    const int b[6] = {oo_rx_blocks_per_cu(), oo_rx_blocks_per_cu_short(), oo_rx_win_blocks_per_cu(),
                      oo_rx_body_blocks_per_cu(), oo_rx_body_blocks_per_cu_gseq(),
                      oo_rx_blocks_per_cu_poll()};
    for (int k = 0; k < 6; ++k) c->bpc[k] = (uint32_t)std::max(0, b[k]);
  }
  apply_tuning(c, nullptr);
  DevTables& T = c->T;
  T.ip4_mask = c->ip4_mask;
  T.ip6_mask = c->ip6_mask;
  T.max_socks = c->max_socks;
  const uint64_t n4 = c->ip4_mask + 1ull, n6 = c->ip6_mask + 1ull;
  // The key index: per protocol up to 2^17 buckets of two entries, up to
  // 2^17 IPv6 entries (a table with more keys than that turns it off).
  T.kx_nb4 = (uint32_t)std::min<uint64_t>(OO_KX_V4_MUL * n4, 1u << OO_KX_LOG2_MAX);
  T.kx_ne6 = (uint32_t)std::min<uint64_t>(OO_KX_V6_MUL * n6, 1u << OO_KX_LOG2_MAX);
  bool ok =
      hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess &&
      hipEventCreateWithFlags(&c->tables_ev, hipEventDisableTiming) == hipSuccess &&
      hipMalloc(&T.slot4, sizeof(Slot4) * n4) == hipSuccess &&
      hipMalloc(&T.rc4, sizeof(int32_t) * n4) == hipSuccess &&
      hipMalloc(&T.occ4, sizeof(uint32_t) * ((n4 + 31) / 32)) == hipSuccess &&
      hipMalloc(&T.slot6, sizeof(Slot6) * n6) == hipSuccess &&
      hipMalloc(&T.occ6, sizeof(uint32_t) * ((n6 + 31) / 32)) == hipSuccess &&
      hipMalloc(&T.socks, sizeof(oo_gpu_rx_sock) * c->max_socks) == hipSuccess &&
      hipMalloc(&T.sockgen, sizeof(uint32_t) * c->max_socks) == hipSuccess &&
      hipMalloc(&c->d_zero, 16u * oo_rx::ZERO_LINES + oo_rx::SINK_BYTES + OO_GPU_RX_MAX_INTF) ==
          hipSuccess &&
      hipMalloc(&c->d_claim, 128u * CLAIM_SETS * oo_rx::CLAIM_LINES) == hipSuccess &&
      hipMemsetAsync(c->d_claim, 0, 128u * CLAIM_SETS * oo_rx::CLAIM_LINES, c->stream) == hipSuccess &&
      hipHostMalloc(&c->h_image_hdr, sizeof(ImageHdr), hipHostMallocDefault) == hipSuccess &&
      hipMemsetAsync(c->d_zero, 0, 16u * oo_rx::ZERO_LINES, c->stream) == hipSuccess &&
      hipMemcpyAsync(c->d_zero + 16u * oo_rx::ZERO_LINES + oo_rx::SINK_BYTES, c->hwport,
                     OO_GPU_RX_MAX_INTF, hipMemcpyHostToDevice, c->stream) == hipSuccess &&
      oo_table_launch_init(&T, c->stream) == 0 &&
      hipMalloc(&T.kx4, oo_table_kx_bytes4(T.kx_nb4)) == hipSuccess &&
      hipMalloc(&T.kx6, oo_table_kx_bytes6(T.kx_ne6)) == hipSuccess &&
      hipMalloc(&T.kx_ok, 128) == hipSuccess && oo_table_launch_kx(&T, c->stream) == 0;
  for (OpStage& st : c->stage)
    ok = ok && hipHostMalloc(&st.h, (sizeof(TableOp) + sizeof(uint32_t)) * OPS_CHUNK,
                             hipHostMallocDefault) == hipSuccess &&
         hipMalloc(&st.d, (sizeof(TableOp) + sizeof(uint32_t)) * OPS_CHUNK) == hipSuccess &&
         hipEventCreateWithFlags(&st.ev, hipEventDisableTiming) == hipSuccess;
  ok = ok && hipHostMalloc(&c->h_len, 128, kGpuWritten) == hipSuccess &&
       hipHostGetDevicePointer(reinterpret_cast<void**>(&c->d_len), c->h_len, 0) == hipSuccess &&
       hipEventCreateWithFlags(&c->len_ev, hipEventDisableTiming) == hipSuccess;
  ok = ok && hipHostMalloc(&c->h_kx_req, 128, kGpuWritten) == hipSuccess &&
       hipHostGetDevicePointer(reinterpret_cast<void**>(&c->d_kx_req), c->h_kx_req, 0) == hipSuccess;
  if (ok) *c->h_kx_req = 0;
  if (ok && cfg->host_stage_bytes && cfg->host_stage_pkts) {
    c->stage_bytes = cfg->host_stage_bytes;
    c->stage_pkts = cfg->host_stage_pkts;
    ok = alloc_host_slots(c) == 0;
  }
  // Every later use of the tables follows the init on the context stream.
  ok = ok && hipStreamSynchronize(c->stream) == hipSuccess;
  if (!ok) {
    free_dev(c);
    delete c;
    return -ENOMEM;
  }
  *out = c;
  return 0;
}

// A context with host memory still registered stays open (-EBUSY): only
// the caller knows when that memory stops being mapped, so the caller
// unregisters it -- before releasing it -- and closes again.  Unregistering
// it here, after the caller may have freed or remapped those pages, is the
// lifetime the round-5 faults pointed at.
int oo_gpu_rx_close(oo_gpu_rx_ctx* c) {
  if (c == nullptr) return 0;
  if (!c->regs.empty()) return -EBUSY;
  if (!has_dev(c)) {
    delete c;
    return 0;
  }
  (void)hipSetDevice(c->device);
  (void)hipDeviceSynchronize();  // every stream the context launched on
  free_dev(c);
  delete c;
  return 0;
}

int oo_gpu_rx_table_insert(oo_gpu_rx_ctx* c, int af, const void* laddr, uint16_t lport,
                           const void* raddr, uint16_t rport, uint8_t proto, int32_t id) {
  if (c == nullptr || laddr == nullptr || id < 0 || (uint32_t)id >= c->max_socks) return -EINVAL;
  int rc;
  if (af == 4)
    rc = ip4_insert(c, id, ld32(laddr), lport, raddr ? ld32(raddr) : 0, rport, proto);
  else if (af == 6)
    rc = ip6_insert(c, id, static_cast<const uint8_t*>(laddr), lport,
                    raddr ? static_cast<const uint8_t*>(raddr) : kZero16, rport, proto);
  else
    return -EINVAL;
  // The device replays the insert, -ENOBUFS included (its raised route
  // counts are part of the table state).
  push_op(c, tuple_op(oo_rx::OP_INSERT, af, laddr, lport, raddr, rport, proto, id));
  ++c->changes;
  return rc;
}

int oo_gpu_rx_table_remove(oo_gpu_rx_ctx* c, int af, const void* laddr, uint16_t lport,
                           const void* raddr, uint16_t rport, uint8_t proto, int32_t id) {
  if (c == nullptr || laddr == nullptr || id < 0 || (uint32_t)id >= c->max_socks) return -EINVAL;
  if (af == 4)
    ip4_remove(c, id, ld32(laddr), lport, raddr ? ld32(raddr) : 0, rport, proto);
  else if (af == 6)
    ip6_remove(c, id, static_cast<const uint8_t*>(laddr), lport,
               raddr ? static_cast<const uint8_t*>(raddr) : kZero16, rport, proto);
  else
    return -EINVAL;
  push_op(c, tuple_op(oo_rx::OP_REMOVE, af, laddr, lport, raddr, rport, proto, id));
  ++c->changes;
  return 0;
}

int oo_gpu_rx_table_lookup(oo_gpu_rx_ctx* c, int af, const void* laddr, uint16_t lport,
                           const void* raddr, uint16_t rport, uint8_t proto) {
  if (c == nullptr || laddr == nullptr) return -EINVAL;
  if (af == 4) return ip4_lookup(c, ld32(laddr), lport, raddr ? ld32(raddr) : 0, rport, proto);
  if (af == 6)
    return ip6_lookup(c, static_cast<const uint8_t*>(laddr), lport,
                      raddr ? static_cast<const uint8_t*>(raddr) : kZero16, rport, proto);
  return -EINVAL;
}

int oo_gpu_rx_table_slot(oo_gpu_rx_ctx* c, int af, uint32_t slot, uint32_t* id_state,
                         int32_t* route_count, uint16_t* lport) {
  if (c == nullptr || id_state == nullptr || route_count == nullptr || lport == nullptr)
    return -EINVAL;
  if (af == 4 && slot <= c->ip4_mask) {
    *id_state = c->ip4[slot].id_state;
    *route_count = c->ip4_ext[slot].route_count;
    *lport = c->ip4_ext[slot].lport;
    return 0;
  }
  if (af == 6 && slot <= c->ip6_mask) {
    *id_state = (uint32_t)c->ip6[slot].id;
    *route_count = c->ip6[slot].route_count;
    *lport = 0;
    return 0;
  }
  return -EINVAL;
}

int oo_gpu_rx_sock_set(oo_gpu_rx_ctx* c, int32_t id, const oo_gpu_rx_sock* s) {
  if (c == nullptr || s == nullptr || id < 0 || (uint32_t)id >= c->max_socks) return -EINVAL;
  c->socks[id] = *s;
  TableOp op;
  memset(&op, 0, sizeof(op));
  op.kind = oo_rx::OP_SOCK;
  op.sock = id;
  op.u.s = *s;
  push_op(c, op);
  ++c->changes;
  return 0;
}

uint64_t oo_gpu_rx_table_gen(const oo_gpu_rx_ctx* c) { return c == nullptr ? 0 : c->changes; }

uint32_t oo_gpu_rx_last_path(const oo_gpu_rx_ctx* c) { return c == nullptr ? 0 : c->last_path; }

int oo_gpu_rx_get_table_stats(oo_gpu_rx_ctx* c, oo_gpu_rx_table_stats* out) {
  if (c == nullptr || out == nullptr) return -EINVAL;
  memset(out, 0, sizeof(*out));
  out->flushes = c->n_flush;
  out->index_rebuilds = c->n_kx_full;
  out->index_updates = c->n_kx_inc;
  if (!has_dev(c)) return 0;
  uint32_t ok = 0;
  if (hipSetDevice(c->device) != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
      hipMemcpy(&ok, c->T.kx_ok, sizeof(ok), hipMemcpyDeviceToHost) != hipSuccess)
    return -EIO;
  out->index_on = ok;
  return 0;
}

int oo_gpu_rx_sync_tables(oo_gpu_rx_ctx* c, void* stream) {
  if (c == nullptr) return -EINVAL;
  if (!has_dev(c)) return -ENODEV;
  if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
  return prepare(c, static_cast<hipStream_t>(stream));
}

int oo_gpu_rx_set_len_hint(oo_gpu_rx_ctx* c, uint32_t mean_frame_len) {
  if (c == nullptr || mean_frame_len > 65535u) return -EINVAL;
  c->len_hint = mean_frame_len;
  return 0;
}

int oo_gpu_rx_stream_done(oo_gpu_rx_ctx* c, void* stream) {
  if (c == nullptr) return -EINVAL;
  if (!has_dev(c)) return 0;
  if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
  hipStream_t s = static_cast<hipStream_t>(stream);
  for (Tracked& t : c->track) {
    if (!t.used || t.gone || t.s != s) continue;
    if (hipEventRecord(t.ev, s) != hipSuccess) return -EIO;
    t.gone = true;  // ev now covers all of s's work; s is never touched again
  }
  // The last table change ran on s: a stream created later may get the same
  // handle, and must still wait for tables_ev.
  if (c->tables_stream == s) c->tables_stream = nullptr;
  return 0;
}

uint64_t oo_gpu_rx_table_image_bytes(const oo_gpu_rx_ctx* c) {
  return c == nullptr ? 0 : image_hdr(c).total;
}

int oo_gpu_rx_table_export(oo_gpu_rx_ctx* c, void* dst, uint64_t bytes, void* stream) {
  if (c == nullptr || dst == nullptr) return -EINVAL;
  const ImageHdr h = image_hdr(c);
  if (bytes < h.total) return -EINVAL;
  if (!has_dev(c)) {
    image_from_mirror(c, static_cast<uint8_t*>(dst));
    return 0;
  }
  if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
  hipStream_t s = static_cast<hipStream_t>(stream);
  Tracked* t = nullptr;
  int rc = prepare(c, s, &t);
  if (rc) return rc;
  uint8_t* d = static_cast<uint8_t*>(dst);
  const uint64_t n4 = c->ip4_mask + 1ull, n6 = c->ip6_mask + 1ull;
  if (hipStreamSynchronize(s) != hipSuccess) return -EIO;  // h_image_hdr reuse
  memcpy(c->h_image_hdr, &h, sizeof(h));
  const bool ok =
      hipMemcpyAsync(d, c->h_image_hdr, sizeof(h), hipMemcpyDefault, s) == hipSuccess &&
      hipMemcpyAsync(d + h.off_slot4, c->T.slot4, sizeof(Slot4) * n4, hipMemcpyDefault, s) ==
          hipSuccess &&
      hipMemcpyAsync(d + h.off_rc4, c->T.rc4, sizeof(int32_t) * n4, hipMemcpyDefault, s) ==
          hipSuccess &&
      hipMemcpyAsync(d + h.off_slot6, c->T.slot6, sizeof(Slot6) * n6, hipMemcpyDefault, s) ==
          hipSuccess &&
      hipMemcpyAsync(d + h.off_socks, c->T.socks, sizeof(oo_gpu_rx_sock) * c->max_socks,
                     hipMemcpyDefault, s) == hipSuccess;
  if (!ok) return -EIO;
  note_launch(t);  // the copies read the tables like a batch
  return 0;
}

int oo_gpu_rx_table_import(oo_gpu_rx_ctx* c, const void* src, uint64_t bytes, void* stream) {
  if (c == nullptr || src == nullptr) return -EINVAL;
  const ImageHdr h = image_hdr(c);
  if (bytes < h.total) return -EINVAL;
  ImageHdr got;
  std::vector<uint8_t> host;
  if (!has_dev(c)) {
    memcpy(&got, src, sizeof(got));
    if (memcmp(&got, &h, sizeof(h)) != 0) return -EINVAL;
    mirror_from_image(c, static_cast<const uint8_t*>(src));
    return 0;
  }
  if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
  hipStream_t s = static_cast<hipStream_t>(stream);
  try {
    host.resize(h.total);
  } catch (...) {
    return -ENOMEM;
  }
  // Setup-time call: the image comes to the host once for the mirror, and
  // the device arrays are copied on the stream after every earlier use.
  clear_ops(c);
  if (order_after_batches(c, s) != 0) return -EIO;
  if (hipMemcpyAsync(host.data(), src, h.total, hipMemcpyDefault, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return -EIO;
  memcpy(&got, host.data(), sizeof(got));
  if (memcmp(&got, &h, sizeof(h)) != 0) return -EINVAL;
  mirror_from_image(c, host.data());
  const uint8_t* d = static_cast<const uint8_t*>(src);
  const uint64_t n4 = c->ip4_mask + 1ull, n6 = c->ip6_mask + 1ull;
  const bool ok =
      hipMemcpyAsync(c->T.slot4, d + h.off_slot4, sizeof(Slot4) * n4, hipMemcpyDefault, s) ==
          hipSuccess &&
      hipMemcpyAsync(c->T.rc4, d + h.off_rc4, sizeof(int32_t) * n4, hipMemcpyDefault, s) ==
          hipSuccess &&
      hipMemcpyAsync(c->T.slot6, d + h.off_slot6, sizeof(Slot6) * n6, hipMemcpyDefault, s) ==
          hipSuccess &&
      hipMemcpyAsync(c->T.socks, d + h.off_socks, sizeof(oo_gpu_rx_sock) * c->max_socks,
                     hipMemcpyDefault, s) == hipSuccess &&
      oo_table_launch_occ(&c->T, s) == 0 && oo_table_launch_kx(&c->T, s) == 0;
  // From here on the mirror holds the image: a failure leaves the device
  // copy unknown.
  Tracked* t = ok ? track_of(c, s) : nullptr;
  if (t == nullptr) {
    c->failed = true;
    return -EIO;
  }
  ++c->tables_gen;
  if (hipEventRecord(c->tables_ev, s) != hipSuccess) {
    c->failed = true;
    return -EIO;
  }
  c->tables_stream = s;
  t->tables_seen = c->tables_gen;
  c->failed = false;  // the whole table state was replaced on both sides
  ++c->changes;
  return 0;
}

// A launch's claim groups: the largest power of two <= gmax with ngroups
// << gshift <= W (every group has a wave).
static void set_groups(KParams& P, uint64_t W, uint32_t gmax, uint32_t gshift) {
  P.gshift = std::min<uint32_t>(gshift, 16u);
  while (P.gshift > 0 && (1ull << P.gshift) > W) --P.gshift;
  P.ngroups = 1;
  while (P.ngroups < gmax && (2ull * P.ngroups << P.gshift) <= W) P.ngroups *= 2;
}

// Dynamic partition of n packets for W waves: full 64-packet tiles, then
// about per_wave tiles of S packets per wave (the last taking what is left,
// at least one packet), so the waves that finish early take the small tiles
// and all end within a small tile of each other.
static void set_tiles_dyn(KParams& P, uint32_t n, uint64_t W, uint32_t S, uint32_t per_wave) {
  const uint64_t tail = W * per_wave * S;
  const uint64_t NA = n > tail ? (n - tail) / 64 : 0;
  const uint64_t NS = S < 64 ? (n - 64 * NA + S - 1) / S : 0;
  P.ntiles = (uint32_t)(NA + NS);
  P.tlo = S;
  P.tstep = 64 - S;
  P.ta = (uint32_t)NA;
  if (S == 64) {  // no tail: plain 64-packet tiles
    P.ntiles = (n + 63) / 64;
    P.tlo = 64;
    P.tstep = 0;
    P.ta = 0;
  }
}

// Whether a launch's batch has the sampled mixed-size profile: the same
// descriptors (address, count, ring position) as the last sampled batch, and
// that sample landed.  No caller hint (a hint names the frames' mean size
// only).  The key names a buffer, not its contents: a caller that refills
// one descriptor buffer gets a fresh sample every kLenResample launches on
// it (sample_lengths), so the choice follows a changed mix within that many
// batches.  (The choice never changes the records, only which kernels run.)
constexpr uint32_t kLenResample = 64;
static bool mixed_sizes(oo_gpu_rx_ctx* c, const KParams& P, uint32_t n) {
  if (c->len_hint != 0 || c->h_len == nullptr) return false;
  if (c->len_desc != static_cast<const void*>(P.desc) || c->len_n != n || c->len_cons != P.ring_cons)
    return false;
  if (c->len_pending && hipEventQuery(c->len_ev) == hipSuccess) {
    const volatile uint32_t* h = c->h_len;
    if (h[6] == c->len_seq) {
      const double cnt = (double)((uint64_t)h[1] << 32 | h[0]);
      const double sum = (double)((uint64_t)h[3] << 32 | h[2]);
      const double sq = (double)((uint64_t)h[5] << 32 | h[4]);
      c->len_mixed = cnt > 0 && sum >= 1024.0 * cnt && sq * cnt >= 1.36 * sum * sum ? 1 : 0;
    }
    c->len_pending = false;
  }
  return c->len_mixed == 1;
}

// After a launch without a hint whose descriptors differ from the last
// sampled ones: a sample of its lengths on s (best effort: a failure only
// leaves the profile unknown).
static void sample_lengths(oo_gpu_rx_ctx* c, const KParams& P, uint32_t n, hipStream_t s) {
  // (only batches the profile can change the choice of: a poll's small
  // batches would pay a launch for nothing)
  // (nor the host path's batches: its two staging slots alternate their
  // descriptor buffers, so every batch would be a new key, sampled and never
  // used -- ADVICE r5; a caller wanting the mixed-size choice there passes
  // a hint)
  if (c->len_hint != 0 || c->h_len == nullptr || c->kmode != 0 || n < (1u << 16) || c->host_batch)
    return;
  const bool same =
      c->len_desc == static_cast<const void*>(P.desc) && c->len_n == n && c->len_cons == P.ring_cons;
  if (same && ++c->len_uses < kLenResample) return;
  c->len_uses = 0;
  c->len_desc = P.desc;
  c->len_n = n;
  c->len_cons = P.ring_cons;
  if (!same) c->len_mixed = -1;  // (a resample keeps the last profile until it lands)
  c->len_pending = oo_launch_len_sample(P.desc, n, P.ring_mask, P.ring_cons, c->d_len, ++c->len_seq, s) == 0 &&
                   hipEventRecord(c->len_ev, s) == hipSuccess;
}

// The split transform (oo_rx_kernel.hip "The split transform"): win_kernel,
// then body_kernel, on s.  The stream's pending-word buffer grows by a new
// allocation (hipMalloc: no wait for the device); the one it replaces may
// still be read by launches in flight, so it is kept until the context
// closes (growth is monotonic: a few buffers at most).  No stream-ordered
// allocator: its memory freed with hipFree at close was a mix the runtime
// does not promise to support.
static int launch_split(oo_gpu_rx_ctx* c, const KParams& base, uint32_t n, Tracked* trk,
                        uint32_t* set, hipStream_t s, bool seq_body) {
  // Mixed sizes (the short-frame class's IMIX, or a sampled profile): the
  // body engine runs per-group job sequences, which idle less of the ring.
  const bool gseq = c->body_engine ? c->body_engine == 2 : seq_body;
  const uint32_t grid_body = gseq ? c->grid_body_gseq : c->grid_body;
  if (trk->pend_n < (uint64_t)n + 64) {
    const uint64_t want = std::max<uint64_t>((uint64_t)n + 64, 1u << 16);
    uint64_t* fresh = nullptr;
    if (hipMalloc(reinterpret_cast<void**>(&fresh), want * 8) != hipSuccess) return -ENOMEM;
    if (trk->pend != nullptr) {
      try {
        c->retired.push_back(trk->pend);
      } catch (...) {
        (void)hipFree(fresh);
        return -ENOMEM;
      }
    }
    trk->pend = fresh;
    trk->pend_n = want;
  }
  KParams B = base, A = base;
  B.pend = A.pend = trk->pend;
  B.flag = A.flag = set + 32u * oo_rx::FLAG_LINE;
  // win_kernel: header-bound tiles, many claims per us (16 groups of
  // 16-wave runs; against 32 groups: config 3 -1.4 %, two reps,
  // profiles/r04/ab_win_claims_c3.log).
  const uint32_t wpb_w = (uint32_t)oo_rx_win_waves_per_block();
  const uint32_t blocks_b =
      std::max<uint32_t>(1, std::min<uint64_t>(((n + 63) / 64 + wpb_w - 1) / wpb_w, c->grid_win));
  const uint64_t WBl = (uint64_t)blocks_b * wpb_w;
  set_groups(B, WBl, c->ngroups_max ? c->ngroups_max : 16u, c->gshift != ~0u ? c->gshift : 4u);
  set_tiles_dyn(B, n, WBl, c->tail_tile, c->tail_per_wave);
  // body_kernel: stream-bound units (64 single-wave groups), a finer tail.
  const uint32_t wpb_b = (uint32_t)oo_rx_body_waves_per_block();
  const uint32_t blocks_a =
      std::max<uint32_t>(1, std::min<uint64_t>(((n + 63) / 64 + wpb_b - 1) / wpb_b, grid_body));
  const uint64_t WA = (uint64_t)blocks_a * (uint32_t)oo_rx_body_waves_per_block();
  A.claim = set + 32u * CLAIM_GROUPS;
  A.claim_next = nullptr;
  set_groups(A, WA, CLAIM_GROUPS, 0u);
  set_tiles_dyn(A, n, WA, c->body_tail, 1);
  A.dyn = B.dyn = 1u;
  if (oo_rx_launch_win(&B, (int)blocks_b, s) != 0) return -EIO;  // nothing ran: the set stays zero
  // win_kernel is queued: it advances this set and zeroes the other, so the
  // stream's next launch takes the other set whether body_kernel follows or not.
  trk->parity ^= 1u;
  if ((gseq ? oo_rx_launch_body_gseq(&A, (int)blocks_a, s) : oo_rx_launch_body(&A, (int)blocks_a, s)) != 0)
    return -EIO;
  return 0;
}

// tx: the TX checksum fill (tx_kernel) instead of the RX transform.
static int launch(oo_gpu_rx_ctx* c, const void* d_frames, uint64_t frames_bytes,
                  const oo_gpu_pkt_desc* d_desc, uint32_t n, oo_gpu_rx_result* d_out,
                  uint32_t* d_ctr, hipStream_t s, bool tx = false,
                  const oo_gpu_xdp_desc* d_ring = nullptr, uint32_t ring_mask = 0,
                  uint32_t cons = 0, int intf_i = 0) {
  KParams P;
  memset(&P, 0, sizeof(P));
  P.frames = static_cast<const uint8_t*>(d_frames);
  P.frames_bytes = frames_bytes;
  P.desc = d_desc;
  P.ring_mask = ~0u;
  if (d_ring != nullptr) {  // both entry layouts are 16 B, offset first
    P.desc = reinterpret_cast<const oo_gpu_pkt_desc*>(d_ring);
    P.ring_mask = ring_mask;
    P.ring_cons = cons;
    P.xdp = 1;
    P.xdp_intf = intf_i;
  }
  P.out = d_out;
  P.counters = d_ctr;
  P.n = n;
  P.ip4_mask = c->ip4_mask;
  P.ip6_mask = c->ip6_mask;
  P.slot4 = c->T.slot4;
  P.occ4 = c->T.occ4;
  P.slot6 = c->T.slot6;
  P.occ6 = c->T.occ6;
  if (c->kx) {
    P.kx4 = c->T.kx4;
    P.kx6 = c->T.kx6;
    P.kx_ok = c->T.kx_ok;
    P.kx_nb4 = c->T.kx_nb4;
    P.kx_ne6 = c->T.kx_ne6;
  }
  P.zero = c->d_zero;
  P.sink = c->d_zero + 16u * oo_rx::ZERO_LINES;
  P.stamps = c->stamps;
  P.hwport = c->d_zero + 16u * oo_rx::ZERO_LINES + oo_rx::SINK_BYTES;
  // Short frames (under 1 KiB of buffer per packet) are bound by the per-tile
  // header and table-lookup chain, not by the body stream: they take the
  // 2-slot-ring rx_kernel, whose smaller LDS footprint fits 12 waves per CU
  // instead of 10 (same-box A/B: config 3 -7 %, config 5 -2 %; config 2
  // +11 %, so long frames keep the 4-slot ring).
  // By the caller's mean-frame-length hint when it gave one (a UMEM of
  // 2048-B chunks says nothing about its frames), else by the buffer bytes
  // per packet (a packed batch).
  const bool short_frames =
      c->len_hint ? c->len_hint < 1024u : P.frames_bytes < 1024ull * n;
  // The stream's own claim counter sets (Tracked): launches on one stream
  // run in order and alternate between the two; each zeroes the other.
  Tracked* trk = track_of(c, s);
  if (trk == nullptr) return -EIO;
  uint32_t* const sets = c->d_claim + 2u * 32u * oo_rx::CLAIM_LINES * track_index(c, trk);
  P.claim = sets + 32u * oo_rx::CLAIM_LINES * trk->parity;
  P.claim_next = sets + 32u * oo_rx::CLAIM_LINES * (trk->parity ^ 1u);
  // The split transform: win_kernel holds the occupancy bitmaps in LDS, so
  // only for tables that fit there (oo_rx_kernel.hip OCC_LDS_MAX4 / _MAX6).
  const bool split_fits = (uint64_t)c->ip4_mask + 1 <= oo_rx::OCC_LDS_MAX4 &&
                          (uint64_t)c->ip6_mask + 1 <= oo_rx::OCC_LDS_MAX6;
  // Auto: batches whose frames fit the 128-B header window (by the hint, or
  // at most 128 buffer bytes per packet) take it from 2^20 packets on --
  // win_kernel alone does their work (config 3 -9 %);
  // body_kernel finds nothing and returns.  Smaller batches keep one launch.
  const bool window_frames =
      c->len_hint ? c->len_hint <= (uint32_t)oo_rx::HB_BYTES : P.frames_bytes <= (uint64_t)oo_rx::HB_BYTES * n;
  // Mixed frame sizes with long frames among them (the sampled profile:
  // mean >= 1 KiB, coefficient of variation >= 0.6 -- config 4's IPv4/TCP
  // 64-9014 B) take the split transform with the sequences body engine:
  // same-box A/B -2.6 % on config 4, while IMIX (mean 362 B, +6 %) and
  // uniform frames (config 2, +57 %) keep one launch
  // (profiles/r05/ab_split_c4_c5.log).
  const bool mixed = !tx && c->kmode == 0 && mixed_sizes(c, P, n);
  const bool split = c->kmode == 3 || (c->kmode == 0 && ((window_frames && n >= (1u << 20)) ||
                                                        (mixed && n >= (1u << 16))));
  if (!tx && split && split_fits && c->grid_win > 0 && c->grid_body > 0 && c->grid_body_gseq > 0) {
    const bool seq_body = short_frames || mixed;
    const int rc = launch_split(c, P, n, trk, P.claim, s, seq_body);  // (flips the parity)
    if (rc != 0) return rc;
    c->last_path = (c->body_engine ? c->body_engine == 2 : seq_body) ? 4u : 3u;
    note_launch(trk);
    sample_lengths(c, P, n, s);
    return 0;
  }
  const bool small = n <= SMALL_N;
  // A poll's batch (at most OO_POLL_MAX packets) takes the poll instance (a
  // 12-slot ring: a tile's frames requested whole with its windows;
  // descriptors in the kernel arguments; its own completion word --
  // oo_rx_kernel.hip "The poll instance").  Same-box A/B, config 2 zero
  // copy: 16 / 64 events -4.5 / -3.9 us per poll, 256 level, 1024 +5 us
  // (profiles/r05/poll_ab_*.jsonl).
  const bool use_poll =
      !tx && c->grid_poll > 0 && (c->kmode == 4 || (c->kmode == 0 && small && n <= OO_POLL_MAX));
  const bool use_short =
      !use_poll && !tx && c->grid_short > 0 && (c->kmode == 2 || (c->kmode == 0 && short_frames));
  const uint32_t wpb = (uint32_t)oo_rx_waves_per_block();
  // A small batch (a poll's worth: at most SMALL_N packets) is cut into tiles
  // of 8 packets, a wave each, statically: its bodies stream in parallel, so
  // the batch takes about one tile's latency -- over PCIe (frames read in
  // place from host memory) one 64-packet tile's 12 KiB in flight would take
  // many round trips.  Larger batches: full 64-packet tiles.
  const uint32_t need = small ? (n + 7) / 8 : (n + 63) / 64;  // waves, a tile each
  const uint32_t blocks = std::max<uint32_t>(
      1, std::min<uint32_t>((need + wpb - 1) / wpb,
                            use_poll ? c->grid_poll : use_short ? c->grid_short : c->grid));
  const uint64_t W = (uint64_t)blocks * wpb;
  // The launch's claim counters (zeroed by the stream's previous launch),
  // one per wave group.  Short frames (under 1 KiB of buffer per packet:
  // header-bound tiles, many claims per us) use 32 groups of eight-block
  // runs, each group spread over all eight XCDs; long frames 64 groups of
  // single waves (same-box A/B).
  set_groups(P, W, c->ngroups_max ? c->ngroups_max : (short_frames ? 32u : CLAIM_GROUPS),
             c->gshift != ~0u ? c->gshift : (short_frames ? 4u : 0u));
  P.dyn = c->dyn && !small ? 1u : 0u;
  if (P.dyn) {
    set_tiles_dyn(P, n, W, c->tail_tile, c->tail_per_wave);
  } else {
    // Static balanced partition: the W waves each take K = ceil(n / (64 W))
    // tiles; NT = W K tiles of tlo or tlo + 8 packets (multiples of 8, at
    // most 64), the last taking the < 8 left over.  Small batches use fewer
    // blocks (and fewer tiles than waves when n < 8 W: no tile is empty).
    const uint64_t K = (n + 64 * W - 1) / (64 * W);
    // W K tiles, but never an empty one (every tile holds at least 8
    // packets, or the whole batch): waves past the last tile have none.
    const uint64_t NT = std::max<uint64_t>(1, std::min<uint64_t>(W * K, n / 8));
    const uint64_t step = c->tstep;
    const uint64_t tlo = std::min<uint64_t>(64 - step, (n / NT) / step * step);
    P.ntiles = (uint32_t)NT;
    P.tlo = (uint32_t)tlo;
    P.ta = (uint32_t)std::min<uint64_t>(NT, (n - tlo * NT) / step);
    P.tstep = (uint32_t)step;
  }
  const int grid = (int)blocks;
  int rc;
  if (use_poll) {
    oo_rx::PollArgs A;
    A.P = P;
    A.done_ctr = P.claim + 32u * oo_rx::FLAG_LINE;
    A.done = n <= OO_POLL_DONE_MAX ? c->poll_done : nullptr;
    A.done_val = c->poll_done_val;
    A.rsvd = 0;
    rc = oo_rx_launch_poll(&A, grid, s);
    if (rc == 0 && A.done != nullptr) c->done_by_kernel = true;
  } else {
    rc = tx ? oo_tx_launch(&P, grid, s)
            : use_short ? oo_rx_launch_short(&P, grid, s) : oo_rx_launch(&P, grid, s);
  }
  if (rc != 0) return -EIO;  // (nothing ran: the set stays zero for the next launch)
  trk->parity ^= 1u;
  if (!tx) {
    note_launch(trk);
    c->last_path = use_poll ? 5u : use_short ? 2u : 1u;
    sample_lengths(c, P, n, s);
  }
  return 0;
}

int oo_gpu_rx_process_dev(oo_gpu_rx_ctx* c, const void* d_frames, uint64_t frames_bytes,
                          const oo_gpu_pkt_desc* d_desc, uint32_t n, oo_gpu_rx_result* d_out,
                          oo_gpu_rx_counters* d_counters, void* stream) {
  if (c == nullptr || (n > 0 && (d_frames == nullptr || d_desc == nullptr || d_out == nullptr)))
    return -EINVAL;
  if (!has_dev(c)) return -ENODEV;
  if (n == 0) return 0;
  if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
  hipStream_t s = static_cast<hipStream_t>(stream);
  int rc = prepare(c, s);
  if (rc) return rc;
  return launch(c, d_frames, frames_bytes, d_desc, n, d_out,
                reinterpret_cast<uint32_t*>(d_counters), s);
}

int oo_gpu_rx_xdp_dev(oo_gpu_rx_ctx* c, const void* d_umem, uint64_t umem_bytes,
                      const oo_gpu_xdp_desc* d_ring, uint32_t ring_mask, uint32_t cons,
                      uint32_t n, int intf_i, oo_gpu_rx_result* d_out,
                      oo_gpu_rx_counters* d_counters, void* stream) {
  static_assert(sizeof(oo_gpu_xdp_desc) == 16 && sizeof(oo_gpu_pkt_desc) == 16,
                "16-B ring entries");
  if (c == nullptr || (ring_mask & (ring_mask + 1u)) != 0 || ring_mask == ~0u ||
      (uint64_t)n > (uint64_t)ring_mask + 1u ||
      (n > 0 && (d_umem == nullptr || d_ring == nullptr || d_out == nullptr)))
    return -EINVAL;
  if (!has_dev(c)) return -ENODEV;
  if (n == 0) return 0;
  if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
  hipStream_t s = static_cast<hipStream_t>(stream);
  int rc = prepare(c, s);
  if (rc) return rc;
  return launch(c, d_umem, umem_bytes, nullptr, n, d_out,
                reinterpret_cast<uint32_t*>(d_counters), s, false, d_ring, ring_mask, cons,
                intf_i);
}

int oo_gpu_rx_xdp_poll(oo_gpu_rx_ctx* c, const void* d_umem, uint64_t umem_bytes,
                       const oo_gpu_xdp_desc* d_ring, uint32_t ring_mask,
                       volatile uint32_t* consumer, const volatile uint32_t* producer,
                       uint32_t max_n, int intf_i, oo_gpu_rx_result* d_out,
                       oo_gpu_rx_counters* d_counters, void* stream) {
  if (consumer == nullptr || producer == nullptr) return -EINVAL;
  const uint32_t cons = *consumer;
  const uint32_t prod = *producer;
  __atomic_thread_fence(__ATOMIC_ACQUIRE);  // entries are read after the producer index
  const uint32_t n = std::min<uint32_t>(prod - cons, max_n);
  int rc = oo_gpu_rx_xdp_dev(c, d_umem, umem_bytes, d_ring, ring_mask, cons, n, intf_i, d_out,
                             d_counters, stream);
  if (rc != 0 || n == 0) return rc;
  if (hipStreamSynchronize(static_cast<hipStream_t>(stream)) != hipSuccess) return -EIO;
  __atomic_thread_fence(__ATOMIC_SEQ_CST);  // the reference's ci_mb() before the store
  *consumer = cons + n;
  return (int)n;
}

int oo_gpu_tx_fill_dev(oo_gpu_rx_ctx* c, void* d_frames, uint64_t frames_bytes,
                       const oo_gpu_pkt_desc* d_desc, uint32_t n, void* stream) {
  if (c == nullptr || (n > 0 && (d_frames == nullptr || d_desc == nullptr))) return -EINVAL;
  if (!has_dev(c)) return -ENODEV;
  if (n == 0) return 0;
  if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
  return launch(c, d_frames, frames_bytes, d_desc, n, nullptr, nullptr,
                static_cast<hipStream_t>(stream), true);
}

// Whole pages only, and none another registration of the process holds:
// the contract Onload's own pools meet (efhw/af_xdp.c:463-500 pins whole
// UMEM pages).  The runtime pins and maps whole pages and looks a host
// address up among the registered ranges when it copies pageable memory, so
// a page shared between two registrations, or between a registration and
// memory the caller hands to other copies, is what DESIGN.md §5 round 6
// names as the fault's condition.  The check and the record are one step
// under the process-wide lock.
int oo_gpu_rx_host_register(oo_gpu_rx_ctx* c, void* p, uint64_t bytes, void** dev_ptr) {
  if (c == nullptr || p == nullptr || bytes == 0) return -EINVAL;
  const uintptr_t page = (uintptr_t)sysconf(_SC_PAGESIZE);
  const uintptr_t lo = reinterpret_cast<uintptr_t>(p);
  if (lo % page != 0 || bytes % page != 0 || lo + bytes < lo) return -EINVAL;
  std::lock_guard<std::mutex> lk(g_reg_mu);
  if (reg_overlaps(lo, lo + bytes)) return -EINVAL;
  // A host-only context keeps the same books (its "device" address of p is
  // p): the contract holds, and is testable, without a GPU.
  const bool dev = has_dev(c);
  void* d = p;
  if (dev) {
    if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
    if (hipHostRegister(p, bytes, hipHostRegisterMapped) != hipSuccess) return -ENOMEM;
    if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
      (void)hipHostUnregister(p);
      return -EIO;
    }
  }
  try {
    c->regs.push_back(HostReg{lo, lo + bytes, d});
    g_reg_pages[lo] = lo + bytes;
  } catch (...) {
    if (!c->regs.empty() && c->regs.back().lo == lo) c->regs.pop_back();
    if (dev) (void)hipHostUnregister(p);
    return -ENOMEM;
  }
  if (dev_ptr) *dev_ptr = d;
  return 0;
}

int oo_gpu_rx_host_registered(const oo_gpu_rx_ctx* c) {
  return c == nullptr ? -EINVAL : (int)c->regs.size();
}

int oo_gpu_rx_host_unregister(oo_gpu_rx_ctx* c, void* p) {
  if (c == nullptr || p == nullptr) return -EINVAL;
  const uintptr_t lo = reinterpret_cast<uintptr_t>(p);
  for (size_t i = 0; i < c->regs.size(); ++i) {
    if (c->regs[i].lo != lo) continue;
    if (!has_dev(c)) {
      std::lock_guard<std::mutex> lk(g_reg_mu);
      g_reg_pages.erase(lo);
      c->regs.erase(c->regs.begin() + (long)i);
      return 0;
    }
    (void)hipSetDevice(c->device);
    // No batch may still read it.
    for (HostSlot& s : c->slot)
      if (s.busy) (void)hipEventSynchronize(s.done);
    // Only a stream that launched since its event was last recorded gets a
    // new one (it may since have been destroyed by a caller that did not
    // call oo_gpu_rx_stream_done); the others' events already
    // cover all their work.
    for (Tracked& t : c->track) {
      if (!t.used) continue;
      hipEvent_t e = t.live ? mark(t) : t.ev;
      if (e != nullptr) (void)hipEventSynchronize(e);
    }
    std::lock_guard<std::mutex> lk(g_reg_mu);
    // A failed unregister leaves the range registered (and the context
    // unclosable): its pages may still be mapped for the device.
    if (hipHostUnregister(p) != hipSuccess) return -EIO;
    g_reg_pages.erase(lo);
    c->regs.erase(c->regs.begin() + (long)i);
    return 0;
  }
  return -ENOENT;
}

// The slot's done word: written by the stream after everything the batch
// enqueued (hipStreamWriteValue32), so seeing it means the records and
// counters have landed.  The waiting thread spins on it -- a host read of its
// own memory, no runtime call -- for up to kSpinNs, then waits on the
// slot's event (a stream that failed to write it, or a long batch).
constexpr int64_t kSpinNs = 50 * 1000 * 1000;
static uint32_t done_word(uint64_t ticket) { return ((uint32_t)ticket & 0x7fffffffu) + 1u; }  // never 0
static bool spin_done(const HostSlot& s) {
  if (s.h_done == nullptr) return false;
  const uint32_t want = done_word(s.ticket);
  const volatile uint32_t* w = s.h_done;
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t i = 0;; ++i) {
    if (*w == want) {
      std::atomic_thread_fence(std::memory_order_acquire);
      return true;
    }
    if ((i & 1023u) == 1023u &&
        std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0)
                .count() > kSpinNs)
      return false;
  }
}

static int complete_slot(oo_gpu_rx_ctx* c, HostSlot& s) {
  if (!spin_done(s) && hipEventSynchronize(s.done) != hipSuccess) {
    s.busy = false;
    return -EIO;
  }
  if (s.copy_out) memcpy(s.out, s.h_out, sizeof(oo_gpu_rx_result) * s.n);
  if (s.delta) memcpy(s.delta, s.h_ctr, sizeof(oo_gpu_rx_counters));
  s.busy = false;
  (void)c;
  return (int)s.n;
}

int oo_gpu_rx_submit(oo_gpu_rx_ctx* c, const void* frames, uint64_t frames_bytes,
                     const oo_gpu_pkt_desc* desc, uint32_t n, oo_gpu_rx_result* out,
                     oo_gpu_rx_counters* delta, uint64_t* ticket) {
  if (c == nullptr || ticket == nullptr ||
      (n > 0 && (frames == nullptr || desc == nullptr || out == nullptr)))
    return -EINVAL;
  if (!has_dev(c)) return -ENODEV;
  if (c->stage_pkts == 0 || n > c->stage_pkts || frames_bytes > c->stage_bytes) return -EINVAL;
  if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
  const uint64_t t = c->next_ticket;
  HostSlot& s = c->slot[t % NSLOT];
  if (s.busy) {  // the slot's previous batch completes first (its results land)
    const int rc = complete_slot(c, s);
    if (rc < 0) return rc;
  }
  hipStream_t st = s.stream;
  // Frames and descriptors: straight from registered memory, otherwise
  // through the slot's pinned staging (so the copies are truly async).
  const void* fsrc = frames;
  const void* dsrc = desc;
  if (n > 0 && !in_reg(c, frames, frames_bytes)) {
    memcpy(s.h_frames, frames, frames_bytes);
    fsrc = s.h_frames;
  }
  if (n > 0 && !in_reg(c, desc, sizeof(oo_gpu_pkt_desc) * n)) {
    memcpy(s.h_desc, desc, sizeof(oo_gpu_pkt_desc) * n);
    dsrc = s.h_desc;
  }
  s.copy_out = n > 0 && !in_reg(c, out, sizeof(oo_gpu_rx_result) * n);
  bool ok = hipMemsetAsync(s.d_ctr, 0, sizeof(oo_gpu_rx_counters), st) == hipSuccess;
  if (n > 0)
    ok = ok &&
         hipMemcpyAsync(s.d_frames, fsrc, frames_bytes, hipMemcpyHostToDevice, st) == hipSuccess &&
         hipMemcpyAsync(s.d_desc, dsrc, sizeof(oo_gpu_pkt_desc) * n, hipMemcpyHostToDevice, st) ==
             hipSuccess;
  if (!ok) return -EIO;
  if (n > 0) {
    int rc = prepare(c, st);
    if (rc == 0) {
      c->host_batch = true;
      rc = launch(c, s.d_frames, frames_bytes, s.d_desc, n, s.d_out, s.d_ctr, st);
      c->host_batch = false;
    }
    if (rc) return rc;
    ok = hipMemcpyAsync(s.copy_out ? s.h_out : out, s.d_out, sizeof(oo_gpu_rx_result) * n,
                        hipMemcpyDeviceToHost, st) == hipSuccess;
  }
  ok = ok && hipMemcpyAsync(s.h_ctr, s.d_ctr, sizeof(oo_gpu_rx_counters), hipMemcpyDeviceToHost,
                            st) == hipSuccess &&
       hipStreamWriteValue32(st, s.d_done, done_word(t), 0) == hipSuccess &&
       hipEventRecord(s.done, st) == hipSuccess;
  if (!ok) return -EIO;
  s.busy = true;
  s.ticket = t;
  s.n = n;
  s.out = out;
  s.delta = delta;
  c->next_ticket = t + 1;
  *ticket = t;
  return 0;
}

int oo_gpu_rx_submit_mapped(oo_gpu_rx_ctx* c, const void* d_frames, uint64_t frames_bytes,
                            const oo_gpu_pkt_desc* d_desc, uint32_t n, oo_gpu_rx_result* d_out,
                            uint64_t* ticket) {
  if (c == nullptr || ticket == nullptr ||
      (n > 0 && (d_frames == nullptr || d_desc == nullptr || d_out == nullptr)))
    return -EINVAL;
  if (!has_dev(c)) return -ENODEV;
  if (c->stage_pkts == 0) return -EINVAL;
  if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
  const uint64_t t = c->next_ticket;
  HostSlot& s = c->slot[t % NSLOT];
  if (s.busy) {
    const int rc = complete_slot(c, s);
    if (rc < 0) return rc;
  }
  hipStream_t st = s.stream;
  bool by_kernel = false;  // the poll instance writes the done word itself
  if (n > 0) {
    int rc = prepare(c, st);
    if (rc == 0) {
      c->poll_done = s.d_done;
      c->poll_done_val = done_word(t);
      c->done_by_kernel = false;
      rc = launch(c, d_frames, frames_bytes, d_desc, n, d_out, nullptr, st);
      by_kernel = rc == 0 && c->done_by_kernel;
      c->poll_done = nullptr;
      c->done_by_kernel = false;
    }
    if (rc) return rc;
  }
  if ((!by_kernel && hipStreamWriteValue32(st, s.d_done, done_word(t), 0) != hipSuccess) ||
      hipEventRecord(s.done, st) != hipSuccess)
    return -EIO;
  s.busy = true;
  s.ticket = t;
  s.n = n;
  s.out = d_out;
  s.delta = nullptr;
  s.copy_out = false;
  c->next_ticket = t + 1;
  *ticket = t;
  return 0;
}

int oo_gpu_rx_wait(oo_gpu_rx_ctx* c, uint64_t ticket) {
  if (c == nullptr) return -EINVAL;
  if (!has_dev(c)) return -ENODEV;
  if (c->stage_pkts == 0) return -EINVAL;
  HostSlot& s = c->slot[ticket % NSLOT];
  if (s.ticket != ticket) return ticket < c->next_ticket ? -ENOENT : -EINVAL;
  if (!s.busy) return -ENOENT;  // already waited for (or completed by a later submit)
  if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
  return complete_slot(c, s);
}

int oo_gpu_rx_batch(oo_gpu_rx_ctx* c, const void* frames, uint64_t frames_bytes,
                    const oo_gpu_pkt_desc* desc, uint32_t n, oo_gpu_rx_result* out,
                    oo_gpu_rx_counters* delta) {
  uint64_t t = 0;
  const int rc = oo_gpu_rx_submit(c, frames, frames_bytes, desc, n, out, delta, &t);
  if (rc) return rc;
  return oo_gpu_rx_wait(c, t);
}

// Diagnostic: device buffer for per-wave phase stamps written by builds with
// -DOO_RX_STAMPS (tools/stamps.py); ignored by the product build.
int oo_gpu_rx_debug_stamps(oo_gpu_rx_ctx* c, void* d_buf) {
  if (c == nullptr) return -EINVAL;
  c->stamps = static_cast<uint64_t*>(d_buf);
  return 0;
}

int oo_gpu_rx_debug_grid(oo_gpu_rx_ctx* c) { return c ? (int)c->grid : -EINVAL; }

#ifdef OO_RX_EXPERIMENTS
// Diagnostic (experiment builds): the key index's arrays copied to host
// memory after pending table changes are applied, and its sizes.
extern "C" int oo_gpu_rx_debug_kx(oo_gpu_rx_ctx* c, void* h4, uint64_t b4, void* h6, uint64_t b6,
                                  uint32_t* nb4_ne6) {
  if (c == nullptr || c->T.kx4 == nullptr) return -EINVAL;
  if (prepare(c, c->stream) != 0) return -EIO;
  nb4_ne6[0] = c->T.kx_nb4;
  nb4_ne6[1] = c->T.kx_ne6;
  if (hipDeviceSynchronize() != hipSuccess) return -EIO;
  if (b4 > oo_table_kx_bytes4(c->T.kx_nb4) || b6 > oo_table_kx_bytes6(c->T.kx_ne6)) return -EINVAL;
  if (hipMemcpy(h4, c->T.kx4, b4, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(h6, c->T.kx6, b6, hipMemcpyDeviceToHost) != hipSuccess)
    return -EIO;
  return 0;
}
#endif

const char* oo_gpu_rx_reason_str(int r) {
  switch (r) {
    case OO_RX_R_DELIVER: return "DELIVER";
    case OO_RX_R_NO_MATCH: return "NO_MATCH";
    case OO_RX_R_IP4_FRAG: return "IP4_FRAG";
    case OO_RX_R_IP4_OPTS_BAD: return "IP4_OPTS_BAD";
    case OO_RX_R_TCP_SCATTERED: return "TCP_SCATTERED";
    case OO_RX_R_SHORT_L2: return "SHORT_L2";
    case OO_RX_R_NOT_IP: return "NOT_IP";
    case OO_RX_R_IP4_LEN: return "IP4_LEN";
    case OO_RX_R_IP4_CSUM: return "IP4_CSUM";
    case OO_RX_R_IP6_LEN: return "IP6_LEN";
    case OO_RX_R_PROTO_OTHER: return "PROTO_OTHER";
    case OO_RX_R_TCP_SHORT: return "TCP_SHORT";
    case OO_RX_R_TCP_CSUM: return "TCP_CSUM";
    case OO_RX_R_UDP_SHORT: return "UDP_SHORT";
    case OO_RX_R_UDP_CSUM: return "UDP_CSUM";
    default: return "?";
  }
}

}  // extern "C"
