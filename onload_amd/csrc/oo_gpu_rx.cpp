// SPDX-License-Identifier: BSD-2-Clause
//
// oo_gpu_rx.cpp -- host side of the C ABI declared in include/oo_gpu_rx.h:
// context lifetime, the filter-table mirror (insert/remove with the
// reference's slot placement, route counts and tombstones), incremental
// upload of the mirror to HBM, and the batch entry points that launch the
// gfx950 kernel in oo_rx_kernel.hip.
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

#include <algorithm>
#include <new>
#include <vector>

#include "oo_rx_device.h"

extern "C" int oo_rx_launch(const oo_rx::KParams* P, int split, int grid, hipStream_t stream);
extern "C" int oo_tx_launch(const oo_rx::KParams* P, int grid, hipStream_t stream);
extern "C" int oo_rx_blocks_per_cu(int split);
extern "C" int oo_rx_waves_per_block(int split);

namespace {

using oo_rx::Ip6Entry;
using oo_rx::KParams;
using oo_rx::Slot4;
using oo_rx::Slot6;

constexpr uint32_t ST_MASK = 0xc0000000u;
constexpr uint32_t ID_MASK = 0x3fffffffu;
constexpr uint32_t ST_PREFERRED = 0x00000000u;
constexpr uint32_t ST_REHASHED = 0x40000000u;
constexpr uint32_t ST_EMPTY = 0x80000000u;
constexpr uint32_t ST_TOMBSTONE = 0xc0000000u;
constexpr int32_t ID6_TOMBSTONE = -1;
constexpr int32_t ID6_EMPTY = -2;

uint32_t env_u32(const char* name, uint32_t dflt) {
  const char* v = getenv(name);
  return (v && *v) ? (uint32_t)strtoul(v, nullptr, 0) : dflt;
}

inline bool occupied(uint32_t st) { return ((~st) & ST_EMPTY & ST_TOMBSTONE) != 0; }

inline uint32_t hash3(uint32_t la, uint32_t lp, uint32_t ra, uint32_t rp, uint32_t proto) {
  uint32_t h = __builtin_bswap32(ra) ^ la ^ ((rp << 16) | lp) ^ proto;
  h ^= h >> 16;
  h ^= h >> 8;
  return h;
}
inline uint32_t hash2(uint32_t la, uint32_t lp, uint32_t ra, uint32_t rp, uint32_t proto) {
  return ((la ^ ra) ^ ((lp << 16) | rp) ^ proto) | 1u;
}
inline uint32_t ld32(const void* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}
inline uint32_t addr_xor(const void* a16) {
  const uint8_t* a = static_cast<const uint8_t*>(a16);
  return ld32(a) ^ ld32(a + 4) ^ ld32(a + 8) ^ ld32(a + 12);
}

// [lo, hi) range of entries changed since the last upload.
struct Dirty {
  uint32_t lo = UINT32_MAX, hi = 0;
  void mark(uint32_t i) {
    lo = std::min(lo, i);
    hi = std::max(hi, i + 1);
  }
  void all(uint32_t n) {
    lo = 0;
    hi = n;
  }
  bool any() const { return hi > lo; }
  void clear() {
    lo = UINT32_MAX;
    hi = 0;
  }
};

struct Entry4 {
  uint32_t id_state, laddr;
};
struct Ext4 {
  int32_t route_count;
  uint16_t lport, pad;
};
static_assert(sizeof(Entry4) == 8 && sizeof(Ext4) == 8, "v4 entry layout");

}  // namespace

struct oo_gpu_rx_ctx {
  int device = 0;
  uint32_t ip4_mask = 0, ip6_mask = 0, max_socks = 0;
  uint8_t hwport[OO_GPU_RX_MAX_INTF];
  std::vector<Entry4> ip4;
  std::vector<Ext4> ip4_ext;
  std::vector<Ip6Entry> ip6;
  std::vector<oo_gpu_rx_sock> socks;
  Dirty dirty_ip4, dirty_ip6, dirty_socks;
  // Device layout (oo_rx_device.h): slot records + not-EMPTY bitmaps, built
  // from the mirror above at sync time.
  std::vector<Slot4> slot4;
  std::vector<uint32_t> occ4;
  std::vector<Slot6> slot6;
  std::vector<uint32_t> occ6;
  Slot4* d_slot4 = nullptr;
  uint32_t* d_occ4 = nullptr;
  Slot6* d_slot6 = nullptr;
  uint32_t* d_occ6 = nullptr;
  uint8_t* d_zero = nullptr;  // oo_rx::ZERO_LINES x 16 B of zeros
  uint32_t grid = 1024;        // resident blocks of rx_kernel
  uint32_t grid_split = 1024;  // resident blocks of rx_split
  uint32_t tstep = 8;                // tile size step (KParams::tstep)
  uint32_t split_min = 0xffffffffu;  // mean bytes per frame from which rx_split runs (never:
                                     // rx_kernel measured as fast or faster on configs 2-5)
  int kernel_force = -1;       // OO_RX_KERNEL: 0 = rx_kernel, 1 = rx_split
  uint64_t* stamps = nullptr;  // diagnostic phase stamps (OO_RX_STAMPS builds)
  // host-path staging
  uint64_t stage_bytes = 0;
  uint32_t stage_pkts = 0;
  uint8_t* d_stage_frames = nullptr;
  oo_gpu_pkt_desc* d_stage_desc = nullptr;
  oo_gpu_rx_result* d_stage_out = nullptr;
  uint32_t* d_stage_ctr = nullptr;
  hipStream_t stream = nullptr;
};

namespace {

// ---- IPv4 mirror: netif_table.c:323-495.
int ip4_insert(oo_gpu_rx_ctx* c, int32_t id, uint32_t la, uint32_t lp, uint32_t ra,
               uint32_t rp, uint32_t proto) {
  uint32_t h1 = hash3(la, lp, ra, rp, proto) & c->ip4_mask;
  const uint32_t h2 = hash2(la, lp, ra, rp, proto);
  const uint32_t first = h1;
  while (occupied(c->ip4[h1].id_state)) {
    ++c->ip4_ext[h1].route_count;
    c->dirty_ip4.mark(h1);
    h1 = (h1 + h2) & c->ip4_mask;
    if (h1 == first) return -ENOBUFS;  // route counts stay raised (:349-376)
  }
  c->ip4[h1].id_state = (h1 == first ? ST_PREFERRED : ST_REHASHED) | ((uint32_t)id & ID_MASK);
  c->ip4[h1].laddr = la;
  c->ip4_ext[h1].lport = (uint16_t)lp;
  c->dirty_ip4.mark(h1);
  return 0;
}

void ip4_remove(oo_gpu_rx_ctx* c, int32_t id, uint32_t la, uint32_t lp, uint32_t ra,
                uint32_t rp, uint32_t proto) {
  const uint32_t h1 = hash3(la, lp, ra, rp, proto) & c->ip4_mask;
  const uint32_t h2 = hash2(la, lp, ra, rp, proto);
  uint32_t i = h1;
  int hops = 0;
  for (;;) {
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
    c->dirty_ip4.mark(i);
    i = (i + h2) & c->ip4_mask;
  }
  c->ip4[i].id_state =
      (c->ip4[i].id_state & ID_MASK) | (c->ip4_ext[i].route_count == 0 ? ST_EMPTY : ST_TOMBSTONE);
  c->dirty_ip4.mark(i);
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
  while (c->ip6[h1].id >= 0) {
    ++c->ip6[h1].route_count;
    c->dirty_ip6.mark(h1);
    h1 = (h1 + h2) & c->ip6_mask;
    if (h1 == first) return -ENOBUFS;
  }
  c->ip6[h1].id = id;
  memcpy(c->ip6[h1].laddr, la, 16);
  c->dirty_ip6.mark(h1);
  return 0;
}

void ip6_remove(oo_gpu_rx_ctx* c, int32_t id, const uint8_t* la, uint32_t lp,
                const uint8_t* ra, uint32_t rp, uint32_t proto) {
  const uint32_t lx = addr_xor(la), rx = addr_xor(ra);
  const uint32_t h1 = hash3(lx, lp, rx, rp, proto) & c->ip6_mask;
  const uint32_t h2 = hash2(lx, lp, rx, rp, proto);
  uint32_t i = h1;
  int hops = 0;
  for (;;) {
    const Ip6Entry& e = c->ip6[i];
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
    Ip6Entry& e = c->ip6[i];
    if (--e.route_count == 0 && e.id == ID6_TOMBSTONE) e.id = ID6_EMPTY;
    c->dirty_ip6.mark(i);
    i = (i + h2) & c->ip6_mask;
  }
  c->ip6[i].id = c->ip6[i].route_count == 0 ? ID6_EMPTY : ID6_TOMBSTONE;
  c->dirty_ip6.mark(i);
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

template <typename T>
int upload(T* dst, const std::vector<T>& src, uint32_t lo, uint32_t hi, hipStream_t s) {
  if (hi <= lo) return 0;
  return hipMemcpyAsync(dst + lo, src.data() + lo, sizeof(T) * (hi - lo), hipMemcpyHostToDevice,
                        s) == hipSuccess
             ? 0
             : -EIO;
}

void free_dev(oo_gpu_rx_ctx* c) {
  if (c->d_slot4) (void)hipFree(c->d_slot4);
  if (c->d_occ4) (void)hipFree(c->d_occ4);
  if (c->d_slot6) (void)hipFree(c->d_slot6);
  if (c->d_occ6) (void)hipFree(c->d_occ6);
  if (c->d_zero) (void)hipFree(c->d_zero);
  if (c->d_stage_frames) (void)hipFree(c->d_stage_frames);
  if (c->d_stage_desc) (void)hipFree(c->d_stage_desc);
  if (c->d_stage_out) (void)hipFree(c->d_stage_out);
  if (c->d_stage_ctr) (void)hipFree(c->d_stage_ctr);
  if (c->stream) (void)hipStreamDestroy(c->stream);
}

// Slot record i from the mirror: the entry, its ext entry and the fields of
// the socket its id names (what netif_table.c:192-231 reads through the id).
void build_slot4(oo_gpu_rx_ctx* c, uint32_t i) {
  Slot4& r = c->slot4[i];
  const Entry4& e = c->ip4[i];
  memset(&r, 0, sizeof(r));
  r.id_state = e.id_state;
  r.laddr = e.laddr;
  r.lport = c->ip4_ext[i].lport;
  const uint32_t id = e.id_state & ID_MASK;
  if ((e.id_state & ST_MASK) != ST_EMPTY && id < c->max_socks) {
    const oo_gpu_rx_sock& k = c->socks[id];
    r.raddr = k.raddr_be32;
    r.rport = k.rport_be16;
    r.proto = k.protocol;
    r.sflags = k.flags;
    r.b2d_vlan = k.bind2dev_vlan;
    r.hwports = k.bind2dev_hwports;
  }
}

void build_slot6(oo_gpu_rx_ctx* c, uint32_t i) {
  Slot6& r = c->slot6[i];
  const Ip6Entry& e = c->ip6[i];
  memset(&r, 0, sizeof(r));
  r.id = e.id;
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
}

int sync_tables(oo_gpu_rx_ctx* c, hipStream_t s) {
  if (c->device < 0) return -ENODEV;
  const bool any = c->dirty_ip4.any() || c->dirty_ip6.any() || c->dirty_socks.any();
  if (!any) return 0;
  // Slots whose socket changed are rebuilt too.
  if (c->dirty_socks.any()) {
    const uint32_t lo = c->dirty_socks.lo, hi = c->dirty_socks.hi;
    for (uint32_t i = 0; i <= c->ip4_mask; ++i) {
      const uint32_t st = c->ip4[i].id_state;
      const uint32_t id = st & ID_MASK;
      if ((st & ST_MASK) != ST_EMPTY && id >= lo && id < hi) c->dirty_ip4.mark(i);
    }
    for (uint32_t i = 0; i <= c->ip6_mask; ++i) {
      const int32_t id = c->ip6[i].id;
      if (id >= 0 && (uint32_t)id >= lo && (uint32_t)id < hi) c->dirty_ip6.mark(i);
    }
    c->dirty_socks.clear();
  }
  int rc = 0;
  if (c->dirty_ip4.any()) {
    const uint32_t lo = c->dirty_ip4.lo, hi = c->dirty_ip4.hi;
    for (uint32_t i = lo; i < hi; ++i) build_slot4(c, i);
    const uint32_t wlo = lo >> 5, whi = ((hi - 1) >> 5) + 1;
    for (uint32_t w = wlo; w < whi; ++w) {
      uint32_t bits = 0;
      for (uint32_t b = 0; b < 32; ++b)
        if ((c->ip4[w * 32 + b].id_state & ST_MASK) != ST_EMPTY) bits |= 1u << b;
      c->occ4[w] = bits;
    }
    rc = upload(c->d_slot4, c->slot4, lo, hi, s);
    if (rc == 0) rc = upload(c->d_occ4, c->occ4, wlo, whi, s);
    c->dirty_ip4.clear();
  }
  if (rc == 0 && c->dirty_ip6.any()) {
    const uint32_t lo = c->dirty_ip6.lo, hi = c->dirty_ip6.hi;
    for (uint32_t i = lo; i < hi; ++i) build_slot6(c, i);
    const uint32_t wlo = lo >> 5, whi = ((hi - 1) >> 5) + 1;
    for (uint32_t w = wlo; w < whi; ++w) {
      uint32_t bits = 0;
      for (uint32_t b = 0; b < 32 && w * 32 + b <= c->ip6_mask; ++b)
        if (c->ip6[w * 32 + b].id != ID6_EMPTY) bits |= 1u << b;
      c->occ6[w] = bits;
    }
    rc = upload(c->d_slot6, c->slot6, lo, hi, s);
    if (rc == 0) rc = upload(c->d_occ6, c->occ6, wlo, whi, s);
    c->dirty_ip6.clear();
  }
  // Pageable sources: make sure the copies consumed the host arrays before
  // the host can modify them again.
  if (rc == 0 && hipStreamSynchronize(s) != hipSuccess) rc = -EIO;
  return rc;
}

}  // namespace

extern "C" {

int oo_gpu_rx_abi_version(void) { return OO_GPU_RX_ABI_VERSION; }

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
    c->ip6.assign(c->ip6_mask + 1, Ip6Entry{ID6_EMPTY, 0, {0, 0, 0, 0}});
    c->socks.assign(c->max_socks, oo_gpu_rx_sock{});
    if (!host_only) {
      c->slot4.assign(c->ip4_mask + 1, Slot4{});
      c->occ4.assign((c->ip4_mask >> 5) + 1, 0u);
      c->slot6.assign(c->ip6_mask + 1, Slot6{});
      c->occ6.assign((c->ip6_mask >> 5) + 1, 0u);
    }
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
    // Persistent grids: every resident block (occupancy query), optionally
    // scaled by OO_RX_GRID_PCT for tuning.
    const uint32_t pct = env_u32("OO_RX_GRID_PCT", 100);
    const int b0 = oo_rx_blocks_per_cu(0), b1 = oo_rx_blocks_per_cu(1);
    if (b0 > 0)
      c->grid = std::max<uint32_t>(1, (uint32_t)(b0 * prop.multiProcessorCount) * pct / 100);
    if (b1 > 0)
      c->grid_split = std::max<uint32_t>(1, (uint32_t)(b1 * prop.multiProcessorCount) * pct / 100);
  }
  c->split_min = env_u32("OO_RX_SPLIT_MIN", c->split_min);
  c->tstep = env_u32("OO_RX_TSTEP", 8) == 1 ? 1 : 8;
  if (const char* k = getenv("OO_RX_KERNEL")) {
    if (!strcmp(k, "split")) c->kernel_force = 1;
    if (!strcmp(k, "lanes")) c->kernel_force = 0;
  }
  bool ok = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess &&
            hipMalloc(&c->d_slot4, sizeof(Slot4) * c->slot4.size()) == hipSuccess &&
            hipMalloc(&c->d_occ4, sizeof(uint32_t) * c->occ4.size()) == hipSuccess &&
            hipMalloc(&c->d_slot6, sizeof(Slot6) * c->slot6.size()) == hipSuccess &&
            hipMalloc(&c->d_occ6, sizeof(uint32_t) * c->occ6.size()) == hipSuccess &&
            hipMalloc(&c->d_zero, 16u * oo_rx::ZERO_LINES + 64u * 32u) == hipSuccess &&
            hipMemset(c->d_zero, 0, 16u * oo_rx::ZERO_LINES) == hipSuccess;
  if (ok && cfg->host_stage_bytes && cfg->host_stage_pkts) {
    c->stage_bytes = cfg->host_stage_bytes;
    c->stage_pkts = cfg->host_stage_pkts;
    ok = hipMalloc(&c->d_stage_frames, c->stage_bytes) == hipSuccess &&
         hipMalloc(&c->d_stage_desc, sizeof(oo_gpu_pkt_desc) * c->stage_pkts) == hipSuccess &&
         hipMalloc(&c->d_stage_out, sizeof(oo_gpu_rx_result) * c->stage_pkts) == hipSuccess &&
         hipMalloc(&c->d_stage_ctr, sizeof(oo_gpu_rx_counters)) == hipSuccess;
  }
  if (!ok) {
    free_dev(c);
    delete c;
    return -ENOMEM;
  }
  c->dirty_ip4.all(c->ip4_mask + 1);
  c->dirty_ip6.all(c->ip6_mask + 1);
  if (sync_tables(c, c->stream) != 0) {
    free_dev(c);
    delete c;
    return -EIO;
  }
  *out = c;
  return 0;
}

void oo_gpu_rx_close(oo_gpu_rx_ctx* c) {
  if (c == nullptr) return;
  if (c->device < 0) {
    delete c;
    return;
  }
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  free_dev(c);
  delete c;
}

int oo_gpu_rx_table_insert(oo_gpu_rx_ctx* c, int af, const void* laddr, uint16_t lport,
                           const void* raddr, uint16_t rport, uint8_t proto, int32_t id) {
  if (c == nullptr || laddr == nullptr || id < 0 || (uint32_t)id >= c->max_socks) return -EINVAL;
  if (af == 4) return ip4_insert(c, id, ld32(laddr), lport, raddr ? ld32(raddr) : 0, rport, proto);
  if (af == 6)
    return ip6_insert(c, id, static_cast<const uint8_t*>(laddr), lport,
                      raddr ? static_cast<const uint8_t*>(raddr) : kZero16, rport, proto);
  return -EINVAL;
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
  c->dirty_socks.mark((uint32_t)id);
  return 0;
}

int oo_gpu_rx_sync_tables(oo_gpu_rx_ctx* c, void* stream) {
  if (c == nullptr) return -EINVAL;
  if (c->device < 0) return -ENODEV;
  if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
  return sync_tables(c, static_cast<hipStream_t>(stream));
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
  P.slot4 = c->d_slot4;
  P.occ4 = c->d_occ4;
  P.slot6 = c->d_slot6;
  P.occ6 = c->d_occ6;
  P.zero = c->d_zero;
  P.sink = c->d_zero + 16u * oo_rx::ZERO_LINES;
  P.stamps = c->stamps;
  memcpy(P.hwport, c->hwport, sizeof(P.hwport));
  // rx_split (parser + streamer waves) for large frames, rx_kernel otherwise;
  // the frame buffer's bytes per descriptor estimate the mean frame size.
  const int split = tx ? 0
                 : c->kernel_force >= 0 ? c->kernel_force
                                        : (frames_bytes >= (uint64_t)c->split_min * n ? 1 : 0);
  // Static balanced partition: the W tile-processing waves (rx_split's
  // streamers) each take K = ceil(n / (64 W)) tiles; NT = W K tiles of tlo or
  // tlo + 8 packets (multiples of 8, at most 64), the last taking the < 8
  // left over.  Small batches use fewer blocks.
  const uint32_t wpb = (uint32_t)oo_rx_waves_per_block(split);
  const uint32_t need = (n + 63) / 64;  // waves if every tile were full
  const uint32_t cap = split ? c->grid_split : c->grid;
  const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>((need + wpb - 1) / wpb, cap));
  const uint64_t W = (uint64_t)blocks * wpb;
  const uint64_t K = (n + 64 * W - 1) / (64 * W);
  const uint64_t NT = W * K;
  const uint64_t step = c->tstep;
  const uint64_t tlo = std::min<uint64_t>(64 - step, (n / NT) / step * step);
  P.ntiles = (uint32_t)NT;
  P.tlo = (uint32_t)tlo;
  P.ta = (uint32_t)std::min<uint64_t>(NT, (n - tlo * NT) / step);
  P.tstep = (uint32_t)step;
  const int grid = (int)blocks;
  if (tx) return oo_tx_launch(&P, grid, s) == 0 ? 0 : -EIO;
  return oo_rx_launch(&P, split, grid, s) == 0 ? 0 : -EIO;
}

int oo_gpu_rx_process_dev(oo_gpu_rx_ctx* c, const void* d_frames, uint64_t frames_bytes,
                          const oo_gpu_pkt_desc* d_desc, uint32_t n, oo_gpu_rx_result* d_out,
                          oo_gpu_rx_counters* d_counters, void* stream) {
  if (c == nullptr || (n > 0 && (d_frames == nullptr || d_desc == nullptr || d_out == nullptr)))
    return -EINVAL;
  if (c->device < 0) return -ENODEV;
  if (n == 0) return 0;
  if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
  hipStream_t s = static_cast<hipStream_t>(stream);
  int rc = sync_tables(c, s);
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
  if (c->device < 0) return -ENODEV;
  if (n == 0) return 0;
  if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
  hipStream_t s = static_cast<hipStream_t>(stream);
  int rc = sync_tables(c, s);
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
  if (c->device < 0) return -ENODEV;
  if (n == 0) return 0;
  if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
  return launch(c, d_frames, frames_bytes, d_desc, n, nullptr, nullptr,
                static_cast<hipStream_t>(stream), true);
}

int oo_gpu_rx_batch(oo_gpu_rx_ctx* c, const void* frames, uint64_t frames_bytes,
                    const oo_gpu_pkt_desc* desc, uint32_t n, oo_gpu_rx_result* out,
                    oo_gpu_rx_counters* delta) {
  if (c == nullptr || (n > 0 && (frames == nullptr || desc == nullptr || out == nullptr)))
    return -EINVAL;
  if (c->device < 0) return -ENODEV;
  if (n > c->stage_pkts || frames_bytes > c->stage_bytes) return -EINVAL;
  if (n == 0) {
    if (delta) memset(delta, 0, sizeof(*delta));
    return 0;
  }
  if (hipSetDevice(c->device) != hipSuccess) return -ENODEV;
  hipStream_t s = c->stream;
  int rc = sync_tables(c, s);
  if (rc) return rc;
  bool ok = hipMemcpyAsync(c->d_stage_frames, frames, frames_bytes, hipMemcpyHostToDevice, s) ==
                hipSuccess &&
            hipMemcpyAsync(c->d_stage_desc, desc, sizeof(oo_gpu_pkt_desc) * n,
                           hipMemcpyHostToDevice, s) == hipSuccess &&
            hipMemsetAsync(c->d_stage_ctr, 0, sizeof(oo_gpu_rx_counters), s) == hipSuccess;
  if (!ok) return -EIO;
  rc = launch(c, c->d_stage_frames, frames_bytes, c->d_stage_desc, n, c->d_stage_out,
              c->d_stage_ctr, s);
  if (rc) return rc;
  ok = hipMemcpyAsync(out, c->d_stage_out, sizeof(oo_gpu_rx_result) * n, hipMemcpyDeviceToHost,
                      s) == hipSuccess;
  if (ok && delta)
    ok = hipMemcpyAsync(delta, c->d_stage_ctr, sizeof(oo_gpu_rx_counters), hipMemcpyDeviceToHost,
                        s) == hipSuccess;
  if (!ok || hipStreamSynchronize(s) != hipSuccess) return -EIO;
  return (int)n;
}

// Diagnostic: device buffer for per-wave phase stamps written by builds with
// -DOO_RX_STAMPS (tools/stamps.py); ignored by the product build.
int oo_gpu_rx_debug_stamps(oo_gpu_rx_ctx* c, void* d_buf) {
  if (c == nullptr) return -EINVAL;
  c->stamps = static_cast<uint64_t*>(d_buf);
  return 0;
}

int oo_gpu_rx_debug_grid(oo_gpu_rx_ctx* c) { return c ? (int)c->grid : -EINVAL; }

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
