// SPDX-License-Identifier: BSD-2-Clause
//
// oo_gpu_rx_group.cpp -- the multi-GPU form of the C ABI (include/oo_gpu_rx.h
// "Multi-GPU group"; SURVEY.md §8(b) "device ids", §8(e)).
//
// Packets are independent and the filter tables are read-only during a
// batch, so a stack's batches spread over the GPUs of one node as
// contiguous shares, one per member, with a replica of the tables on every
// member and no collective on the data path.  What moves between members:
//  * table changes -- every replica applies the same ops in the same order
//    (the mirror's and the device's placement are deterministic, so the
//    replicas stay byte-identical, return codes included: oof applies its
//    deferred ops at one serialisation point the same way,
//    oof_interface.c:184-217);
//  * the records, gathered into one array after a batch, and the counters,
//    summed.
// Two shapes:
//  * in one process (oo_gpu_rx_group_open): members on a list of devices
//    (a device may repeat), driven by the calling thread -- Onload's stack
//    lives in one process;
//  * across processes, one per GPU (oo_gpu_rx_group_join): this process's
//    one member, RCCL over xGMI between the ranks (librccl, loaded when the
//    first group joins) for the table image, the ops and the records.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <dlfcn.h>
#include <errno.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <vector>

#include "oo_rx_device.h"

namespace {

// librccl entry points (dlopen: the library is needed only by a group that
// joins across processes).
struct Rccl {
  void* h = nullptr;
  ncclResult_t (*get_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*bcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t,
                        hipStream_t) = nullptr;
  ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*allreduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                            hipStream_t) = nullptr;
  ncclResult_t (*group_start)(void) = nullptr;
  ncclResult_t (*group_end)(void) = nullptr;
};

Rccl* rccl() {
  static Rccl r;
  static bool tried = false;
  if (tried) return r.h ? &r : nullptr;
  tried = true;
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (h == nullptr) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
  if (h == nullptr) return nullptr;
  bool ok = true;
  auto sym = [&](auto& fn, const char* name) {
    fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
    ok = ok && fn != nullptr;
  };
  sym(r.get_id, "ncclGetUniqueId");
  sym(r.init_rank, "ncclCommInitRank");
  sym(r.destroy, "ncclCommDestroy");
  sym(r.bcast, "ncclBroadcast");
  sym(r.send, "ncclSend");
  sym(r.recv, "ncclRecv");
  sym(r.allreduce, "ncclAllReduce");
  sym(r.group_start, "ncclGroupStart");
  sym(r.group_end, "ncclGroupEnd");
  if (!ok) {
    dlclose(h);
    return nullptr;
  }
  r.h = h;
  return &r;
}

// One table change as it travels to the other ranks (join shape): the
// arguments of oo_gpu_rx_table_insert / _remove / oo_gpu_rx_sock_set, and
// the return code rank 0 got for it (a replica that gets another has
// diverged).  96 B.
struct GroupOp {
  uint8_t kind;  // 1 insert, 2 remove, 3 socket
  uint8_t af, proto, raddr_any;
  uint16_t lport, rport;
  int32_t sock;
  int32_t rc;
  uint8_t laddr[16], raddr[16];
  oo_gpu_rx_sock s;
};
static_assert(sizeof(GroupOp) == 96, "group op layout");

// The op broadcast goes in fixed chunks through staging allocated at the
// join: share_ops allocates nothing, so no rank can fail between two
// collectives that the others enter.  A 16-B header (the count and rank 0's
// flags) travels first; then ceil(count / kOpsPerChunk) body broadcasts,
// the same number on every rank because every rank acts on the broadcast
// count.
constexpr uint64_t kOpsPerChunk = 8192;  // 768 KiB of ops
constexpr uint64_t kOpsHdr = 16;
constexpr uint32_t kOpsLost = 1;  // rank 0 could not queue an op: re-share the tables

}  // namespace

// The join shape's collectives, on host words or on the group's data
// memory (device memory over RCCL; host memory over a caller transport).
// Every method enters its collective on every rank, whatever failed before
// it locally, and reports a local failure by its return code.
struct Xport {
  virtual ~Xport() {}
  // rank 0's `bytes` at host address h to every rank's h (bytes <= the
  // op staging: kOpsHdr + one chunk)
  virtual int bcast_words(void* h, uint64_t bytes) = 0;
  // element-wise maximum over the ranks of n host words, in place
  virtual int max_words(uint32_t* h, uint32_t n) = 0;
  // rank 0's image at the group's staging p to every rank's
  virtual int bcast_image(void* p, uint64_t bytes) = 0;
  // every rank's `bytes` at src to rank 0's dst in rank order (bytes_of:
  // every rank's bytes, known to every rank)
  virtual int gather(const void* src, uint64_t bytes, void* dst, const uint64_t* bytes_of) = 0;
  // the per-reason counters at p summed over the ranks, in place
  virtual int sum_counters(uint32_t* p) = 0;
  // the work the calls above queued has completed
  virtual int sync() = 0;
  virtual bool rccl() const = 0;
};

struct oo_gpu_rx_group {
  std::vector<oo_gpu_rx_ctx*> m;  // local members
  std::vector<int32_t> dev;       // their devices
  // join shape
  uint32_t rank = 0, nranks = 1;
  Xport* x = nullptr;             // the collectives (RCCL or a caller transport)
  std::vector<GroupOp> ops;       // rank 0's changes since the last share_ops
  bool ops_lost = false;          // a change rank 0 applied but could not queue
  std::vector<GroupOp> h_ops;     // host staging for one chunk
  void* img = nullptr;            // staging for the table image (device, or host)
  bool img_host = false;
  uint64_t img_bytes = 0;
};

namespace {

int apply_op(oo_gpu_rx_ctx* c, const GroupOp& o) {
  const void* ra = o.raddr_any ? nullptr : o.raddr;
  switch (o.kind) {
    case 1: return oo_gpu_rx_table_insert(c, o.af, o.laddr, o.lport, ra, o.rport, o.proto, o.sock);
    case 2: return oo_gpu_rx_table_remove(c, o.af, o.laddr, o.lport, ra, o.rport, o.proto, o.sock);
    case 3: return oo_gpu_rx_sock_set(c, o.sock, &o.s);
    default: return -EINVAL;
  }
}

// Applies one change to every local member in order (and queues it for
// the other ranks in the join shape): the first member's return code; the
// replicas agree, and a member that does not is reported as -EIO.
int group_change(oo_gpu_rx_group* g, GroupOp o) {
  if (g->m.empty()) return -EINVAL;
  if (g->x != nullptr && g->rank != 0) return -EPERM;  // rank 0 owns the tables
  const int rc = apply_op(g->m[0], o);
  for (size_t i = 1; i < g->m.size(); ++i)
    if (apply_op(g->m[i], o) != rc) return -EIO;
  if (g->x != nullptr) {
    o.rc = rc;
    try {
      g->ops.push_back(o);
    } catch (...) {
      g->ops_lost = true;  // the next share_ops fails on every rank
      return -ENOMEM;
    }
  }
  return rc;
}

GroupOp tuple_change(uint8_t kind, int af, const void* laddr, uint16_t lport, const void* raddr,
                     uint16_t rport, uint8_t proto, int32_t id) {
  GroupOp o;
  memset(&o, 0, sizeof(o));
  o.kind = kind;
  o.af = (uint8_t)af;
  o.proto = proto;
  o.lport = lport;
  o.rport = rport;
  o.sock = id;
  const size_t n = af == 6 ? 16 : 4;
  if (laddr) memcpy(o.laddr, laddr, n);
  if (raddr) memcpy(o.raddr, raddr, n);
  else o.raddr_any = 1;
  return o;
}

// RCCL over xGMI: host words staged through device memory allocated at the
// join (no collective call allocates, so none fails between two
// collectives the other ranks enter), the data buffers used in place.
struct RcclXport final : Xport {
  Rccl* r = nullptr;
  ncclComm_t comm = nullptr;
  uint32_t rank = 0, nranks = 1;
  hipStream_t s = nullptr;  // the current call's stream
  void* d_words = nullptr;  // kOpsHdr + one chunk of ops

  ~RcclXport() override {
    if (d_words) (void)hipFree(d_words);
    if (comm) (void)r->destroy(comm);
  }
  int bcast_words(void* h, uint64_t bytes) override {
    int err = 0;
    if (rank == 0 && hipMemcpyAsync(d_words, h, bytes, hipMemcpyHostToDevice, s) != hipSuccess)
      err = -EIO;
    if (r->bcast(d_words, d_words, bytes, ncclUint8, 0, comm, s) != ncclSuccess) err = -EIO;
    if (hipMemcpyAsync(h, d_words, bytes, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      err = -EIO;
    return err;
  }
  int max_words(uint32_t* h, uint32_t n) override {
    int err = 0;
    if (hipMemcpyAsync(d_words, h, 4ull * n, hipMemcpyHostToDevice, s) != hipSuccess) err = -EIO;
    if (r->allreduce(d_words, d_words, n, ncclUint32, ncclMax, comm, s) != ncclSuccess) err = -EIO;
    if (hipMemcpyAsync(h, d_words, 4ull * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      err = -EIO;
    return err;
  }
  int bcast_image(void* p, uint64_t bytes) override {
    return r->bcast(p, p, bytes, ncclUint8, 0, comm, s) == ncclSuccess ? 0 : -EIO;
  }
  int gather(const void* src, uint64_t bytes, void* dst, const uint64_t* bytes_of) override {
    if (r->group_start() != ncclSuccess) return -EIO;
    ncclResult_t e = ncclSuccess;
    if (rank == 0) {
      uint64_t at = 0;
      for (uint32_t k = 0; k < nranks; ++k) {
        const uint64_t b = bytes_of[k];
        if (k == 0 && nranks > 1) {
          // rank 0's own records: a copy on the stream
          if (b && dst != src &&
              hipMemcpyAsync(dst, src, b, hipMemcpyDefault, s) != hipSuccess)
            e = ncclSystemError;
        } else if (b) {
          // the other ranks' (and, in a group of one, rank 0's own through a
          // send to itself)
          const ncclResult_t er =
              r->recv(static_cast<uint8_t*>(dst) + at, b, ncclUint8, (int)k, comm, s);
          if (e == ncclSuccess) e = er;
        }
        at += b;
      }
    }
    if ((rank != 0 || nranks == 1) && bytes > 0) {
      const ncclResult_t er = r->send(src, bytes, ncclUint8, 0, comm, s);
      if (e == ncclSuccess) e = er;
    }
    const ncclResult_t e2 = r->group_end();
    return (e == ncclSuccess && e2 == ncclSuccess) ? 0 : -EIO;
  }
  int sum_counters(uint32_t* p) override {
    return r->allreduce(p, p, OO_RX_R_COUNT, ncclUint32, ncclSum, comm, s) == ncclSuccess ? 0 : -EIO;
  }
  int sync() override { return hipStreamSynchronize(s) == hipSuccess ? 0 : -EIO; }
  bool rccl() const override { return true; }
};

// A caller's transport (oo_gpu_rx_group_transport) on host memory.
struct HostXport final : Xport {
  oo_gpu_rx_group_transport t;
  int bcast_words(void* h, uint64_t bytes) override { return t.bcast(t.arg, h, bytes); }
  int max_words(uint32_t* h, uint32_t n) override { return t.max_u32(t.arg, h, n); }
  int bcast_image(void* p, uint64_t bytes) override { return t.bcast(t.arg, p, bytes); }
  int gather(const void* src, uint64_t bytes, void* dst, const uint64_t* bytes_of) override {
    return t.gather(t.arg, src, bytes, dst, bytes_of);
  }
  int sum_counters(uint32_t* p) override { return t.sum_u32(t.arg, p, OO_RX_R_COUNT); }
  int sync() override { return 0; }
  bool rccl() const override { return false; }
};

void group_free(oo_gpu_rx_group* g) {
  for (oo_gpu_rx_ctx* c : g->m) (void)oo_gpu_rx_close(c);
  if (g->img) {
    if (g->img_host) free(g->img);
    else (void)hipFree(g->img);
  }
  delete g->x;
  delete g;
}

// Every rank learns whether any rank failed (a local error as a flag): the
// one word all ranks decide on before a collective that only some would
// otherwise enter.  1: some rank failed; 0: none; < 0: the agreement itself
// failed here (the communicator is unusable; the caller abandons the group).
int agree(oo_gpu_rx_group* g, int local_err) {
  uint32_t w = local_err != 0 ? 1u : 0u;
  const int e = g->x->max_words(&w, 1);
  return e != 0 ? e : (int)w;
}

// The join-shape checks shared by the collectives: one local member and a
// communicator or transport (a group opened in one process has neither).
int join_shape(oo_gpu_rx_group* g, void* stream) {
  if (g == nullptr || g->m.size() != 1) return -EINVAL;
  if (g->x == nullptr) return g->nranks == 1 ? 1 : -ENOSYS;
  if (g->x->rccl()) {
    if (hipSetDevice(g->dev[0]) != hipSuccess) return -ENODEV;
    static_cast<RcclXport*>(g->x)->s = static_cast<hipStream_t>(stream);
  }
  return 0;
}

}  // namespace

extern "C" {

int oo_gpu_rx_group_open(oo_gpu_rx_group** out, const oo_gpu_rx_cfg* cfg, const int32_t* devices,
                         uint32_t n) {
  if (out == nullptr || cfg == nullptr || devices == nullptr || n == 0 || n > 64) return -EINVAL;
  *out = nullptr;
  oo_gpu_rx_group* g = new (std::nothrow) oo_gpu_rx_group();
  if (g == nullptr) return -ENOMEM;
  try {
    for (uint32_t i = 0; i < n; ++i) {
      oo_gpu_rx_cfg c = *cfg;
      c.device = devices[i];
      oo_gpu_rx_ctx* ctx = nullptr;
      const int rc = oo_gpu_rx_open(&ctx, &c);
      if (rc != 0) {
        group_free(g);
        return rc;
      }
      g->m.push_back(ctx);
      g->dev.push_back(devices[i]);
    }
  } catch (...) {
    group_free(g);
    return -ENOMEM;
  }
  *out = g;
  return 0;
}

int oo_gpu_rx_group_rccl_id(void* id) {
  if (id == nullptr) return -EINVAL;
  Rccl* r = rccl();
  if (r == nullptr) return -ENOSYS;
  ncclUniqueId u;
  if (r->get_id(&u) != ncclSuccess) return -EIO;
  static_assert(sizeof(u) == OO_GPU_RX_GROUP_ID_BYTES, "RCCL unique id size");
  memcpy(id, &u, sizeof(u));
  return 0;
}

int oo_gpu_rx_group_join(oo_gpu_rx_group** out, const oo_gpu_rx_cfg* cfg, uint32_t rank,
                         uint32_t nranks, const void* id) {
  if (out == nullptr || cfg == nullptr || id == nullptr || nranks == 0 || rank >= nranks ||
      cfg->device < 0)
    return -EINVAL;
  *out = nullptr;
  Rccl* r = rccl();
  if (r == nullptr) return -ENOSYS;
  oo_gpu_rx_group* g = nullptr;
  int rc = oo_gpu_rx_group_open(&g, cfg, &cfg->device, 1);
  if (rc != 0) return rc;
  g->rank = rank;
  g->nranks = nranks;
  // Every buffer a collective call needs is allocated here, before the
  // communicator exists: the collective calls allocate nothing, so a rank
  // never leaves one of them early on a local allocation failure.
  g->img_bytes = oo_gpu_rx_table_image_bytes(g->m[0]);
  RcclXport* x = new (std::nothrow) RcclXport();
  if (x == nullptr) {
    group_free(g);
    return -ENOMEM;
  }
  g->x = x;
  x->r = r;
  x->rank = rank;
  x->nranks = nranks;
  try {
    g->h_ops.resize(kOpsPerChunk);
  } catch (...) {
    group_free(g);
    return -ENOMEM;
  }
  if (hipSetDevice(cfg->device) != hipSuccess) {
    group_free(g);
    return -ENODEV;
  }
  if (hipMalloc(&x->d_words, kOpsHdr + sizeof(GroupOp) * kOpsPerChunk) != hipSuccess ||
      hipMalloc(&g->img, g->img_bytes) != hipSuccess) {
    group_free(g);
    return -ENOMEM;
  }
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  if (r->init_rank(&x->comm, (int)nranks, u, (int)rank) != ncclSuccess) {
    x->comm = nullptr;
    group_free(g);
    return -EIO;
  }
  *out = g;
  return 0;
}

int oo_gpu_rx_group_join_transport(oo_gpu_rx_group** out, const oo_gpu_rx_cfg* cfg, uint32_t rank,
                                   uint32_t nranks, const oo_gpu_rx_group_transport* t) {
  if (out == nullptr || cfg == nullptr || t == nullptr || nranks == 0 || rank >= nranks ||
      cfg->device >= 0 || t->bcast == nullptr || t->max_u32 == nullptr || t->sum_u32 == nullptr ||
      t->gather == nullptr)
    return -EINVAL;
  *out = nullptr;
  oo_gpu_rx_group* g = nullptr;
  int rc = oo_gpu_rx_group_open(&g, cfg, &cfg->device, 1);
  if (rc != 0) return rc;
  g->rank = rank;
  g->nranks = nranks;
  g->img_bytes = oo_gpu_rx_table_image_bytes(g->m[0]);
  HostXport* x = new (std::nothrow) HostXport();
  if (x == nullptr) {
    group_free(g);
    return -ENOMEM;
  }
  x->t = *t;
  g->x = x;
  g->img_host = true;
  g->img = malloc(g->img_bytes);
  try {
    g->h_ops.resize(kOpsPerChunk);
  } catch (...) {
    group_free(g);
    return -ENOMEM;
  }
  if (g->img == nullptr) {
    group_free(g);
    return -ENOMEM;
  }
  *out = g;
  return 0;
}

int oo_gpu_rx_group_close(oo_gpu_rx_group* g) {
  if (g == nullptr) return 0;
  // (nothing is closed while a member holds registered host memory: see
  // oo_gpu_rx_close)
  for (oo_gpu_rx_ctx* c : g->m)
    if (oo_gpu_rx_host_registered(c) > 0) return -EBUSY;
  group_free(g);
  return 0;
}

uint32_t oo_gpu_rx_group_size(const oo_gpu_rx_group* g) { return g ? (uint32_t)g->m.size() : 0; }

uint32_t oo_gpu_rx_group_rank(const oo_gpu_rx_group* g) { return g ? g->rank : 0; }

oo_gpu_rx_ctx* oo_gpu_rx_group_member(oo_gpu_rx_group* g, uint32_t i) {
  return (g && i < g->m.size()) ? g->m[i] : nullptr;
}

int oo_gpu_rx_group_table_insert(oo_gpu_rx_group* g, int af, const void* laddr, uint16_t lport,
                                 const void* raddr, uint16_t rport, uint8_t proto, int32_t id) {
  if (g == nullptr || laddr == nullptr || (af != 4 && af != 6)) return -EINVAL;
  return group_change(g, tuple_change(1, af, laddr, lport, raddr, rport, proto, id));
}

int oo_gpu_rx_group_table_remove(oo_gpu_rx_group* g, int af, const void* laddr, uint16_t lport,
                                 const void* raddr, uint16_t rport, uint8_t proto, int32_t id) {
  if (g == nullptr || laddr == nullptr || (af != 4 && af != 6)) return -EINVAL;
  return group_change(g, tuple_change(2, af, laddr, lport, raddr, rport, proto, id));
}

int oo_gpu_rx_group_sock_set(oo_gpu_rx_group* g, int32_t id, const oo_gpu_rx_sock* s) {
  if (g == nullptr || s == nullptr) return -EINVAL;
  GroupOp o;
  memset(&o, 0, sizeof(o));
  o.kind = 3;
  o.sock = id;
  o.s = *s;
  return group_change(g, o);
}

int oo_gpu_rx_group_split(const oo_gpu_rx_group* g, const oo_gpu_pkt_desc* desc, uint32_t n,
                          uint32_t parts, uint32_t* first) {
  if (g == nullptr || first == nullptr || parts == 0 || (n > 0 && desc == nullptr)) return -EINVAL;
  // The algorithmic bytes of a packet: its frame, its descriptor and its
  // record (DESIGN.md §2 "Rooflines"); every share gets about total / parts.
  uint64_t total = 0;
  for (uint32_t i = 0; i < n; ++i) total += (uint64_t)desc[i].len + 48u;
  first[0] = 0;
  uint64_t acc = 0;
  uint32_t k = 1;
  for (uint32_t i = 0; i < n && k < parts; ++i) {
    acc += (uint64_t)desc[i].len + 48u;
    while (k < parts && acc * parts >= total * k) first[k++] = i + 1;
  }
  while (k <= parts) first[k++] = n;
  return 0;
}

int oo_gpu_rx_group_process(oo_gpu_rx_group* g, const oo_gpu_rx_shard* shards) {
  if (g == nullptr || shards == nullptr) return -EINVAL;
  for (size_t i = 0; i < g->m.size(); ++i) {
    const oo_gpu_rx_shard& s = shards[i];
    const int rc = oo_gpu_rx_process_dev(g->m[i], s.d_frames, s.frames_bytes, s.d_desc, s.n,
                                         s.d_out, s.d_counters, s.stream);
    if (rc != 0) return rc;
  }
  return 0;
}

int oo_gpu_rx_group_gather(oo_gpu_rx_group* g, const oo_gpu_rx_shard* shards,
                           oo_gpu_rx_result* dst, oo_gpu_rx_counters* counters) {
  if (g == nullptr || shards == nullptr) return -EINVAL;
  uint64_t at = 0;
  for (size_t i = 0; i < g->m.size(); ++i) {
    const oo_gpu_rx_shard& s = shards[i];
    if (g->dev[i] < 0 || hipSetDevice(g->dev[i]) != hipSuccess) return -ENODEV;
    hipStream_t st = static_cast<hipStream_t>(s.stream);
    if (dst != nullptr && s.n > 0 &&
        hipMemcpyAsync(dst + at, s.d_out, sizeof(oo_gpu_rx_result) * s.n, hipMemcpyDefault, st) !=
            hipSuccess)
      return -EIO;
    at += s.n;
  }
  if (counters != nullptr) memset(counters, 0, sizeof(*counters));
  for (size_t i = 0; i < g->m.size(); ++i) {
    const oo_gpu_rx_shard& s = shards[i];
    if (hipSetDevice(g->dev[i]) != hipSuccess ||
        hipStreamSynchronize(static_cast<hipStream_t>(s.stream)) != hipSuccess)
      return -EIO;
    if (counters != nullptr && s.d_counters != nullptr) {
      oo_gpu_rx_counters c;
      if (hipMemcpy(&c, s.d_counters, sizeof(c), hipMemcpyDefault) != hipSuccess) return -EIO;
      for (int k = 0; k < OO_RX_R_COUNT; ++k) counters->by_reason[k] += c.by_reason[k];
    }
  }
  return 0;
}

// The join shape's collectives.  Every rank enters every collective of a
// call: their number depends only on values every rank holds -- broadcast
// from rank 0, or agreed on by a one-word maximum (agree) before any rank
// could decide alone to stop -- and a local failure after the last of them
// is reported by the return code, never by leaving early.  A group opened in
// one process has no communicator: there they do nothing (one member is its
// own rank 0).  A joined group of one rank runs the same RCCL calls as a
// larger one (broadcasts and all-reduce of one rank, the gather as a
// send/receive pair to itself).

int oo_gpu_rx_group_share_tables(oo_gpu_rx_group* g, void* stream) {
  const int sh = join_shape(g, stream);
  if (sh != 0) return sh > 0 ? 0 : sh;
  oo_gpu_rx_ctx* c = g->m[0];
  int rc = 0;
  if (g->rank == 0) rc = oo_gpu_rx_table_export(c, g->img, g->img_bytes, stream);
  // (rank 0 joins the broadcast even when its export failed)
  const int e = g->x->bcast_image(g->img, g->img_bytes);
  if (rc == 0) rc = e;
  if (rc == 0) rc = g->x->sync();
  // No replica imports unless every rank has the image: the staging may
  // still hold the previous share's, which would pass the import's checks.
  const int any = agree(g, rc);
  if (any < 0) return any;
  if (any) return rc ? rc : -EIO;
  if (g->rank != 0) {
    rc = oo_gpu_rx_table_import(c, g->img, g->img_bytes, stream);
    if (rc == 0) rc = g->x->sync();
  } else {
    g->ops.clear();  // rank 0's changes so far are in the image
    g->ops_lost = false;
  }
  return rc;
}

int oo_gpu_rx_group_share_ops(oo_gpu_rx_group* g, void* stream) {
  const int sh = join_shape(g, stream);
  if (sh != 0) return sh > 0 ? 0 : sh;
  int err = 0;
  auto fail = [&err](int e) {
    if (err == 0) err = e;
  };
  // The header: the count and rank 0's flags.  Then every rank learns
  // whether every rank has it before any enters the body broadcasts.
  uint64_t hdr[2] = {g->rank == 0 ? (uint64_t)g->ops.size() : 0,
                     g->rank == 0 && g->ops_lost ? kOpsLost : 0u};
  const int eh = g->x->bcast_words(hdr, kOpsHdr);
  const int any = agree(g, eh);
  if (any < 0) return any;
  if (any) return eh ? eh : -EIO;  // some rank has no count: none goes on (rank 0 keeps its ops)
  const uint64_t cnt = hdr[0];
  for (uint64_t at = 0; at < cnt; at += kOpsPerChunk) {
    const uint64_t k = std::min<uint64_t>(kOpsPerChunk, cnt - at);
    const uint64_t bytes = sizeof(GroupOp) * k;
    if (g->rank == 0) memcpy(g->h_ops.data(), g->ops.data() + at, bytes);
    if (g->x->bcast_words(g->h_ops.data(), bytes) != 0) {
      fail(-EIO);
      continue;
    }
    if (g->rank == 0) {
      // rank 0 applied these at its calls: what came back must be them
      if (memcmp(g->h_ops.data(), g->ops.data() + at, bytes) != 0) fail(-EIO);
    } else {
      for (uint64_t i = 0; i < k; ++i) {
        const GroupOp& o = g->h_ops[i];
        if (apply_op(g->m[0], o) != o.rc) fail(-EIO);  // this replica diverged
      }
    }
  }
  if (g->rank == 0) {
    g->ops.clear();
    g->ops_lost = false;
  }
  if (hdr[1] & kOpsLost) fail(-EIO);  // every rank: share the tables again
  return err ? err : (int)cnt;
}

int oo_gpu_rx_group_gather_rccl(oo_gpu_rx_group* g, const oo_gpu_rx_result* d_out, uint32_t n,
                                oo_gpu_rx_result* d_dst, const uint32_t* counts, void* stream) {
  if (g == nullptr || g->m.size() != 1 || (n > 0 && d_out == nullptr)) return -EINVAL;
  if (g->x == nullptr) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (g->nranks != 1) return -ENOSYS;
    if (hipSetDevice(g->dev[0]) != hipSuccess) return -ENODEV;
    if (d_dst != nullptr && n > 0 && d_dst != d_out &&
        hipMemcpyAsync(d_dst, d_out, sizeof(oo_gpu_rx_result) * n, hipMemcpyDefault, s) != hipSuccess)
      return -EIO;
    return 0;
  }
  const int sh = join_shape(g, stream);
  if (sh != 0) return sh;
  // Rank 0's counts (and whether it has a destination) to every rank; each
  // checks its own entry, and all agree before any record moves: a count
  // that does not match its rank's n is -EINVAL on every rank, where it
  // would otherwise hang or truncate the gather.
  std::vector<uint32_t> w;
  std::vector<uint64_t> bytes_of;
  try {
    w.assign(g->nranks + 1u, 0u);
    bytes_of.assign(g->nranks, 0u);
  } catch (...) {
    w.clear();
  }
  int local = 0;
  if (w.empty() || 4ull * w.size() > kOpsHdr + sizeof(GroupOp) * kOpsPerChunk) {
    // (no words to exchange: still enter both collectives, with one word)
    uint32_t dummy[1] = {0};
    (void)g->x->bcast_words(dummy, 4);
    local = 2;
  } else {
    if (g->rank == 0) {
      w[0] = (d_dst != nullptr && counts != nullptr) ? 1u : 0u;
      if (counts != nullptr)
        for (uint32_t k = 0; k < g->nranks; ++k) w[1 + k] = counts[k];
    }
    if (g->x->bcast_words(w.data(), 4ull * w.size()) != 0) local = 2;
    else if (w[0] == 0 || w[1 + g->rank] != n) local = 1;
  }
  uint32_t v = (uint32_t)local;
  const int ea = g->x->max_words(&v, 1);
  if (ea != 0) return ea;
  if (v != 0) return v == 1 ? -EINVAL : -EIO;
  for (uint32_t k = 0; k < g->nranks; ++k) bytes_of[k] = sizeof(oo_gpu_rx_result) * (uint64_t)w[1 + k];
  return g->x->gather(d_out, sizeof(oo_gpu_rx_result) * (uint64_t)n, d_dst, bytes_of.data());
}

int oo_gpu_rx_group_sum_counters(oo_gpu_rx_group* g, oo_gpu_rx_counters* d_counters, void* stream) {
  if (g == nullptr || g->m.size() != 1 || d_counters == nullptr) return -EINVAL;
  const int sh = join_shape(g, stream);
  if (sh != 0) return sh > 0 ? 0 : sh;
  return g->x->sum_counters(d_counters->by_reason);
}

int oo_gpu_rx_group_uses_rccl(const oo_gpu_rx_group* g) { return g && g->x && g->x->rccl() ? 1 : 0; }

}  // extern "C"
