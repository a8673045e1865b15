/* SPDX-License-Identifier: BSD-2-Clause */
/*
 * oo_rx_poll.c -- batched software-RX branch of ci_netif_poll_evq over
 * liboo_gpu_rx.  See include/oo_rx_poll.h for the contract; each step below
 * names the reference code whose behaviour it keeps.
 *
 * One call of oo_rx_poll_evs takes its events evs_per_poll at a time
 * ("chunks"), two chunks in flight:
 *   1. classify each event of a chunk (netif_event.c:1715-1742 RX branch,
 *      :1843 discard_rx_multi_pkts): transform / release / other_ev, and
 *      count the per-event stats the loop keeps (rx_evs, rx_discard_*);
 *   2. describe the frames to transform -- in place in the packet-buffer
 *      pool when it is registered with the device (zero copy: the kernel
 *      reads them over PCIe), else gathered into a registered buffer -- and
 *      submit the chunk's device batch;
 *   3. while the next chunk's batch runs, wait for this one and walk its
 *      records in event order, dispatching each through the callback table
 *      and counting what the replaced code counts.
 */
#include "oo_rx_poll.h"

#include <errno.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

enum { W_TRANSFORM = 0, W_RELEASE = 1, W_OTHER = 2 };

/* One chunk's buffers; two of them alternate. */
struct chunk {
  oo_gpu_pkt_desc*  desc;      /* evs_per_poll descriptors (registered)     */
  oo_gpu_rx_result* rec;       /* evs_per_poll records (registered)         */
  void*             d_desc;    /* their device addresses (mapped)           */
  void*             d_rec;
  uint8_t*          pack;      /* gathered frames (gather mode, registered) */
  void*             d_pack;
  uint32_t*         ev_of;     /* transform slot -> event index             */
  uint8_t*          what;      /* per event: W_*                            */
  const oo_rx_poll_ev* evs;
  uint32_t          n, m;      /* events, frames to transform               */
  int               busy;      /* a device batch was submitted              */
  uint64_t          ticket;
  oo_rx_poll_stats  st;        /* the chunk's counters (land with it)       */
};

struct oo_rx_poll {
  oo_gpu_rx_ctx*   gpu;
  oo_rx_poll_cfg   cfg;
  oo_rx_poll_ops   ops;
  uint64_t         pack_bytes;
  int              mapped;     /* chunk buffers registered: submit_mapped    */
  int              zero_copy;  /* the pool is registered: frames in place    */
  void*            d_pool;     /* its device address                         */
  struct chunk     ch[2];
};

static uint64_t up64(uint64_t x) { return (x + 63u) & ~(uint64_t)63u; }

static uint16_t be16_at(const uint8_t* p) { return (uint16_t)(p[0] << 8 | p[1]); }

static uint32_t be32_at(const uint8_t* p)
{
  return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}

/* The buffers the device maps (descriptors, records, gathered frames):
 * whole pages of their own, from mmap, so no other allocation of the
 * process ever shares a page with a registered range (DESIGN.md §5 round 5,
 * the faults).  Zeroed. */
static uint64_t page_bytes(uint64_t bytes)
{
  return ((bytes ? bytes : 1) + 4095) & ~(uint64_t)4095;
}

static void* alloc_pages(uint64_t bytes)
{
  void* p = mmap(NULL, page_bytes(bytes), PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS,
                 -1, 0);
  return p == MAP_FAILED ? NULL : p;
}

static void free_pages(void* p, uint64_t bytes)
{
  if( p != NULL )
    munmap(p, page_bytes(bytes));
}

/* Registers the whole pages of one of the shim's own buffers (alloc_pages)
 * with the device; 1 and *d set on success. */
static int reg(oo_gpu_rx_ctx* gpu, void* p, uint64_t bytes, void** d)
{
  return oo_gpu_rx_host_register(gpu, p, page_bytes(bytes), d) == 0;
}

static void chunk_free(oo_rx_poll* p, struct chunk* c)
{
  if( c->d_desc )
    oo_gpu_rx_host_unregister(p->gpu, c->desc);
  if( c->d_rec )
    oo_gpu_rx_host_unregister(p->gpu, c->rec);
  if( c->d_pack )
    oo_gpu_rx_host_unregister(p->gpu, c->pack);
  free_pages(c->pack, p->pack_bytes);
  free_pages(c->desc, sizeof(oo_gpu_pkt_desc) * (uint64_t)p->cfg.evs_per_poll);
  free_pages(c->rec, sizeof(oo_gpu_rx_result) * (uint64_t)p->cfg.evs_per_poll);
  free(c->ev_of);
  free(c->what);
}

void oo_rx_poll_close(oo_rx_poll* p)
{
  int i;
  if( p == NULL )
    return;
  for( i = 0; i < 2; ++i ) {
    if( p->ch[i].busy )
      (void)oo_gpu_rx_wait(p->gpu, p->ch[i].ticket);
    chunk_free(p, &p->ch[i]);
  }
  if( p->d_pool )
    oo_gpu_rx_host_unregister(p->gpu, (void*)p->cfg.pkt_bufs);
  free(p);
}

static int chunk_alloc(oo_rx_poll* p, struct chunk* c)
{
  const uint32_t n = p->cfg.evs_per_poll;
  c->desc = alloc_pages(sizeof(oo_gpu_pkt_desc) * (uint64_t)n);
  c->rec = alloc_pages(sizeof(oo_gpu_rx_result) * (uint64_t)n);
  c->ev_of = malloc(sizeof(uint32_t) * (uint64_t)n);
  c->what = malloc(n);
  if( !p->zero_copy )
    c->pack = alloc_pages(p->pack_bytes);
  if( !c->desc || !c->rec || !c->ev_of || !c->what || (!p->zero_copy && !c->pack) )
    return -ENOMEM;
  return 0;
}

int oo_rx_poll_open(oo_rx_poll** out, oo_gpu_rx_ctx* gpu, const oo_rx_poll_cfg* cfg,
                    const oo_rx_poll_ops* ops)
{
  oo_rx_poll* p;
  uint32_t n;
  int i;
  if( out == NULL || gpu == NULL || cfg == NULL || ops == NULL )
    return -EINVAL;
  *out = NULL;
  n = cfg->evs_per_poll;
  if( n == 0 || n > OO_RX_POLL_MAX_EVS || cfg->buf_size == 0 ||
      (cfg->buf_size & (cfg->buf_size - 1)) != 0 || cfg->buf_size > 65536 ||
      (cfg->pkt_bufs == NULL && cfg->pkt_bufs_bytes != 0) ||
      (cfg->flags & ~(uint32_t)(OO_RX_POLL_ZERO_COPY | OO_RX_POLL_CROSSOVER)) != 0 )
    return -EINVAL;
  if( ops->post_future == NULL || ops->full_handler == NULL ||
      ops->pkt_handler == NULL || ops->release == NULL || ops->other_ev == NULL )
    return -EINVAL;
  p = calloc(1, sizeof(*p));
  if( p == NULL )
    return -ENOMEM;
  p->gpu = gpu;
  p->cfg = *cfg;
  p->ops = *ops;
  /* Zero copy: the kernel reads each frame where the NIC put it.  If the
   * pool cannot be registered the shim gathers instead. */
  if( (cfg->flags & OO_RX_POLL_ZERO_COPY) && cfg->pkt_bufs_bytes > 0 &&
      oo_gpu_rx_host_register(gpu, (void*)cfg->pkt_bufs, cfg->pkt_bufs_bytes, &p->d_pool) == 0 )
    p->zero_copy = 1;  /* (a pool that is not whole pages: -EINVAL, gathered) */
  /* A transformed frame lies inside its buffer (frame_of): a gather buffer
   * of evs_per_poll 64-B-aligned buffers holds any chunk. */
  p->pack_bytes = (uint64_t)n * up64(cfg->buf_size);
  p->mapped = 1;
  for( i = 0; i < 2; ++i ) {
    struct chunk* c = &p->ch[i];
    if( chunk_alloc(p, c) != 0 ) {
      oo_rx_poll_close(p);
      return -ENOMEM;
    }
    /* Registered chunk buffers: the batch reads descriptors (and gathered
     * frames) and writes records in place, nothing is staged. */
    if( !reg(gpu, c->desc, sizeof(oo_gpu_pkt_desc) * (uint64_t)n, &c->d_desc) ||
        !reg(gpu, c->rec, sizeof(oo_gpu_rx_result) * (uint64_t)n, &c->d_rec) ||
        (!p->zero_copy && !reg(gpu, c->pack, p->pack_bytes, &c->d_pack)) )
      p->mapped = 0;
  }
  if( !p->mapped && p->zero_copy ) {
    /* Frames in place need mapped descriptors and records. */
    oo_gpu_rx_host_unregister(gpu, (void*)cfg->pkt_bufs);
    p->d_pool = NULL;
    p->zero_copy = 0;
    for( i = 0; i < 2; ++i )
      if( (p->ch[i].pack = alloc_pages(p->pack_bytes)) == NULL ) {
        oo_rx_poll_close(p);
        return -ENOMEM;
      }
  }
  *out = p;
  return 0;
}

int oo_rx_poll_zero_copy(const oo_rx_poll* p)
{
  return p == NULL ? -EINVAL : p->zero_copy;
}

/* The frame of an event, or NULL if it does not lie inside its buffer of the
 * pool (such an event is not the shim's to take: ADVICE r2, a frame running
 * past its buffer would overrun a gather slot). */
static const uint8_t* frame_of(const oo_rx_poll* p, const oo_rx_poll_ev* e)
{
  uint64_t off = (uint64_t)e->rq_id * p->cfg.buf_size + e->ofs;
  if( (uint32_t)e->ofs + e->len > p->cfg.buf_size || off > p->cfg.pkt_bufs_bytes ||
      e->len > p->cfg.pkt_bufs_bytes - off )
    return NULL;
  return (const uint8_t*)p->cfg.pkt_bufs + off;
}

/* Step 1: what the poll loop does with an event before any transform
 * (netif_event.c:1715-1742 plain RX, :1131-1191 discard).  A plain RX event
 * the shim does not take goes back to the caller's loop, which counts its
 * rx_evs (:1718) itself. */
static int classify(const oo_rx_poll* p, const oo_rx_poll_ev* e, oo_rx_poll_stats* st)
{
  const int whole = (e->flags & (OO_RX_EV_SOP | OO_RX_EV_CONT)) == OO_RX_EV_SOP;
  if( e->discard == 0 ) {
    if( !p->cfg.sw_verify || !whole || frame_of(p, e) == NULL )
      return W_OTHER;                                      /* reference branch */
    ++st->rx_evs;                                          /* :1718 */
    return W_TRANSFORM;
  }
  /* discard_rx_multi_pkts: the class counter (:1164-1172) ... */
  if( e->discard & OO_RX_DISCARD_ETH_LEN_ERR )
    ++st->rx_discard_len_err;
  else if( e->discard & OO_RX_DISCARD_ETH_FCS_ERR )
    ++st->rx_discard_crc_bad;
  else if( e->discard & (OO_RX_DISCARD_L3_CSUM_ERR | OO_RX_DISCARD_L4_CSUM_ERR) )
    ++st->rx_discard_csum_bad;
  else
    ++st->rx_discard_other;
  /* ... and handle_rx_csum_bad only for the checksum class, never for a
   * multi-buffer packet (:1155-1162); the rest is released (:1175-1183). */
  if( (e->discard & (OO_RX_DISCARD_L3_CSUM_ERR | OO_RX_DISCARD_L4_CSUM_ERR |
                     OO_RX_DISCARD_L3_CLASS_OTHER)) && whole && frame_of(p, e) )
    return W_TRANSFORM;
  return W_RELEASE;
}

/* The drop counters of handle_rx_csum_bad itself (netif_event.c:1014-1128). */
static void count_drop(const oo_gpu_rx_result* r, oo_rx_poll_stats* st)
{
  switch( r->reason ) {
  case OO_RX_R_SHORT_L2:   /* :1031 -- counted as IPv4 whatever the type */
  case OO_RX_R_IP4_LEN:    /* :1048 */
  case OO_RX_R_IP4_CSUM:   /* :1055 */
    ++st->in_hdr_errs;
    break;
  case OO_RX_R_IP6_LEN:    /* :1069 */
    ++st->in6_hdr_errs;
    break;
  case OO_RX_R_UDP_CSUM:   /* :1116 */
    ++st->udp_in_errs;
    break;
  default:                 /* NOT_IP, PROTO_OTHER, TCP_*, UDP_SHORT: log only */
    break;
  }
}

/* Whether the record resolves a future socket: IPv4 TCP decided in lookup
 * stage 1 (ci_tcp_handle_rx_pre_future: the full 4-tuple lookup only,
 * tcp_rx.h:150-184), or IPv4 UDP whose two lookup stages together hold
 * exactly one socket (ci_udp_handle_rx_pre_future, udp_internal.h:58-103:
 * ci_udp_rx_deliver_to_future keeps walking after the first match and gives
 * up on a second one, :41-52; stage 2 runs whenever stage 1 did not give up,
 * :93-97).  The device record carries the deciding stage's count (nmatch)
 * and, for a stage-1 single match, whether stage 2 matches too
 * (OO_RX_F_UDP_S2). */
static int resolves_future(const oo_gpu_rx_result* r)
{
  if( (r->flags & OO_RX_F_IP6) || r->reason != OO_RX_R_DELIVER )
    return 0;
  if( r->proto == 6 )
    return r->stage == 1;
  return r->proto == 17 && r->nmatch == 1 && !(r->flags & OO_RX_F_UDP_S2);
}

/* Step 3 for a handled record (handle_rx_csum_bad returned 1):
 * __handle_rx_pkt -> handle_rx_pkt (:250-451) up to the transport call, then
 * the future seam. */
static void dispatch(oo_rx_poll* p, uint32_t id, const uint8_t* frame,
                     const oo_gpu_rx_result* r, oo_rx_poll_stats* st)
{
  const int is6 = (r->flags & OO_RX_F_IP6) != 0;
  int future = 0;
  if( r->reason == OO_RX_R_IP4_FRAG || r->reason == OO_RX_R_IP4_OPTS_BAD ) {
    /* not_fast (:293-303): handle_rx_pkt's slow path passes the packet to
     * the kernel and keeps its own counters (in_recvs, in_discards,
     * rx_discard_ip_options_bad, ...). */
    ++st->n_pkt_handler;
    p->ops.pkt_handler(p->ops.arg, id, frame, r);
    return;
  }
  if( is6 ) {
    ++st->in6_recvs;                                       /* :384 */
  }
  else {
    const unsigned pre_l3 = (r->flags & OO_RX_F_VLAN) ? 18u : 14u;
    ++st->in_recvs;                                        /* :282 */
    if( r->l4_off > pre_l3 + 20u )
      ++st->ip_options;                                    /* :181 */
    future = resolves_future(r);
  }
  if( future ) {
    oo_rx_poll_future f;
    const uint8_t* l4 = frame + r->l4_off;
    memset(&f, 0, sizeof(f));
    f.sock = r->sock;
    f.l4_off = r->l4_off;
    f.ip_paylen = r->ip_paylen;
    if( r->proto == 6 ) {
      f.hash = r->hash3;                                   /* rxp.hash   */
      f.seq = be32_at(l4 + 4);                             /* tcp_rx.h:177 */
      f.ack = be32_at(l4 + 8);                             /* tcp_rx.h:178 */
      f.pay_len = r->ip_paylen;                            /* :175 */
    }
    else {
      f.pay_len = (uint32_t)be16_at(l4 + 4) - 8u;          /* udp_internal.h:76-80 */
    }
    if( p->ops.post_future(p->ops.arg, id, frame, r, &f) == 0 ) {
      ++st->n_future;
      if( r->proto == 6 )
        ++st->tcp_in_segs;                                 /* tcp_rx.h:182 */
      else
        ++st->udp_in_dgrams;                               /* udp_internal.h:99 */
    }
    else {
      /* The socket cannot take it now: the NULL-future fallback. */
      ++st->n_future_declined;
      ++st->n_full;
      p->ops.full_handler(p->ops.arg, id, frame, r);
    }
  }
  else {
    ++st->n_full;
    p->ops.full_handler(p->ops.arg, id, frame, r);
  }
  if( is6 )
    ++st->in6_delivers;                                    /* :394 / :400 */
  else
    ++st->in_delivers;                                     /* :327 / :332 */
}

/* The crossover's cost model (oo_rx_poll.h): whether the device batch of m
 * frames and `bytes` frame bytes costs less than the caller's per-event
 * path.  The defaults are tools/poll_bench's fit on an MI355X box
 * (profiles/r06/poll_latency_product.jsonl): the
 * per-event path 21.3 ns per frame + 0.121 ns per byte on one host core; a
 * device batch (the poll instance up to 256 frames) ~17.4 us fixed
 * (launch, PCIe and HBM round trips, the completion word) + 15 ns per
 * frame, + 0.019 ns per byte read in place (zero copy) or 0.075 ns per byte
 * gathered (the host memcpy). */
static int gpu_pays(const oo_rx_poll* p, uint64_t m, uint64_t bytes)
{
  const oo_rx_poll_cfg* c = &p->cfg;
  const uint64_t cpu_pkt = c->cpu_pkt_ps ? c->cpu_pkt_ps : 21300;
  const uint64_t cpu_byte = c->cpu_byte_ps ? c->cpu_byte_ps : 121;
  const uint64_t fixed = (uint64_t)(c->gpu_fixed_ns ? c->gpu_fixed_ns : 17400) * 1000u;
  const uint64_t gpu_pkt = c->gpu_pkt_ps ? c->gpu_pkt_ps : 15000;
  const uint64_t gpu_byte = c->gpu_byte_ps ? c->gpu_byte_ps : (p->zero_copy ? 19 : 75);
  return fixed + m * gpu_pkt + bytes * gpu_byte < m * cpu_pkt + bytes * cpu_byte;
}

/* Steps 1-2 for the chunk evs[0..n): classify, describe, submit.  0 or
 * -errno (the chunk is then not in flight and nothing was counted). */
static int chunk_submit(oo_rx_poll* p, struct chunk* c, const oo_rx_poll_ev* evs, uint32_t n,
                        const oo_rx_poll_stats* base)
{
  uint32_t i, m = 0;
  uint64_t at = 0, total = 0;
  int rc;
  c->evs = evs;
  c->n = n;
  c->busy = 0;
  c->st = *base;
  if( p->cfg.flags & OO_RX_POLL_CROSSOVER ) {
    /* Priced first with every event transformed: the device's side of the
     * model only gains with more frames, so a chunk that loses even then
     * goes back at once, unclassified. */
    for( i = 0; i < n; ++i )
      total += evs[i].len;
    if( !gpu_pays(p, n, total) ) {
      for( i = 0; i < n; ++i )
        c->what[i] = W_OTHER;
      c->st.n_handback += n;
      c->m = 0;
      return 0;
    }
    total = 0;
  }
  for( i = 0; i < n; ++i ) {
    c->what[i] = (uint8_t)classify(p, &evs[i], &c->st);
    if( c->what[i] == W_TRANSFORM ) {
      total += evs[i].len;
      ++m;
    }
  }
  c->m = m;
  if( m == 0 )
    return 0;
  if( (p->cfg.flags & OO_RX_POLL_CROSSOVER) && !gpu_pays(p, m, total) ) {
    /* Cheaper one event at a time: the whole chunk goes back, uncounted. */
    for( i = 0; i < n; ++i )
      c->what[i] = W_OTHER;
    c->st = *base;
    c->st.n_handback += n;
    c->m = 0;
    return 0;
  }
  for( i = 0, m = 0; i < n; ++i ) {
    const oo_rx_poll_ev* e = &evs[i];
    if( c->what[i] == W_TRANSFORM ) {
      oo_gpu_pkt_desc* d = &c->desc[m];
      if( p->zero_copy ) {
        d->frame_off = (uint64_t)e->rq_id * p->cfg.buf_size + e->ofs;
      }
      else {
        /* frame_of bounds the frame by its buffer, and the gather buffer
         * holds evs_per_poll 64-B-aligned buffers */
        if( at + e->len > p->pack_bytes )
          return -EINVAL;
        memcpy(c->pack + at, frame_of(p, e), e->len);
        d->frame_off = at;
        at += up64(e->len);
      }
      d->len = e->len;
      d->intf_i = e->intf_i;
      d->rsvd = 0;
      c->ev_of[m++] = i;
    }
  }
  if( p->zero_copy ) {
    /* The frames sit in their 2048-B packet buffers, so the buffer bytes per
     * packet say nothing of their length: the poll's mean length picks the
     * kernel instance for this launch (and is cleared after it). */
    (void)oo_gpu_rx_set_len_hint(p->gpu, (uint32_t)(total / m) ? (uint32_t)(total / m) : 1u);
    rc = oo_gpu_rx_submit_mapped(p->gpu, p->d_pool, p->cfg.pkt_bufs_bytes, c->d_desc, m,
                                 c->d_rec, &c->ticket);
    (void)oo_gpu_rx_set_len_hint(p->gpu, 0);
  }
  else {
    /* the gathered frames are packed, but their mean length names the
     * kernel instance without a look at the buffer */
    (void)oo_gpu_rx_set_len_hint(p->gpu, (uint32_t)(total / m) ? (uint32_t)(total / m) : 1u);
    if( p->mapped )
      rc = oo_gpu_rx_submit_mapped(p->gpu, c->d_pack, at, c->d_desc, m, c->d_rec, &c->ticket);
    else
      rc = oo_gpu_rx_submit(p->gpu, c->pack, at, c->desc, m, c->rec, NULL, &c->ticket);
    (void)oo_gpu_rx_set_len_hint(p->gpu, 0);
  }
  if( rc < 0 )
    return rc;
  c->busy = 1;
  ++c->st.n_batches;
  return 0;
}

/* Step 3: wait for the chunk's batch, then dispatch every event in order.
 * The chunk's counters are added to *st only if its batch ran.  A callback
 * that changes the tables (a filter inserted on an accept, removed on a
 * close, next to ci_netif_filter_insert / _remove) while transformed events
 * of the chunk are still to come: the reference loop, one event after
 * another, runs those on the new tables, so they are transformed again
 * (counted in n_resubmit; their first records are discarded, nothing was
 * dispatched from them). */
static int chunk_complete(oo_rx_poll* p, struct chunk* c, oo_rx_poll_stats* st)
{
  uint32_t i, m = 0;
  uint64_t gen;
  if( c->busy ) {
    int rc = oo_gpu_rx_wait(p->gpu, c->ticket);
    c->busy = 0;
    if( rc < 0 )
      return rc;
  }
  gen = oo_gpu_rx_table_gen(p->gpu);
  for( i = 0; i < c->n; ++i ) {
    const oo_rx_poll_ev* e = &c->evs[i];
    if( c->what[i] == W_OTHER ) {
      ++c->st.n_other;
      p->ops.other_ev(p->ops.arg, e);
    }
    else if( c->what[i] == W_RELEASE ) {
      ++c->st.n_release;
      p->ops.release(p->ops.arg, e->rq_id, frame_of(p, e), NULL);
    }
    else {
      const oo_gpu_rx_result* r = &c->rec[m++];
      const uint8_t* frame = frame_of(p, e);
      if( r->reason >= OO_RX_R_DROP_BASE ) {
        count_drop(r, &c->st);
        ++c->st.n_release;
        p->ops.release(p->ops.arg, e->rq_id, frame, r);
      }
      else {
        if( e->discard ) {         /* the discard path's double count, :1189-1190 */
          ++c->st.rx_evs;
          ++c->st.rx_sw_csum_pass;
        }
        dispatch(p, e->rq_id, frame, r, &c->st);
      }
    }
    if( m < c->m && oo_gpu_rx_table_gen(p->gpu) != gen ) {
      /* The rest of the chunk becomes a chunk of its own, transformed on the
       * new tables.  Its events were classified (and counted) already: only
       * the batch or the hand-back is added to the counters. */
      const oo_rx_poll_stats saved = c->st;
      const oo_rx_poll_ev* rest = c->evs + i + 1;
      const uint32_t nrest = c->n - i - 1;
      oo_rx_poll_stats cls;
      uint64_t handed;
      uint32_t j;
      int rc;
      /* what the first classification of the rest counted (in saved) */
      memset(&cls, 0, sizeof(cls));
      for( j = 0; j < nrest; ++j )
        (void)classify(p, &rest[j], &cls);
      rc = chunk_submit(p, c, rest, nrest, &saved);
      handed = c->st.n_handback - saved.n_handback;
      c->st = saved;
      if( handed ) {
        /* the rest goes to other_ev: the caller's loop counts it itself */
        uint64_t* a = (uint64_t*)&c->st;
        const uint64_t* b = (const uint64_t*)&cls;
        for( j = 0; j < sizeof(oo_rx_poll_stats) / sizeof(uint64_t); ++j )
          a[j] -= b[j];
      }
      c->st.n_handback += handed;
      ++c->st.n_resubmit;
      if( rc < 0 )
        return rc;
      if( c->busy ) {
        ++c->st.n_batches;
        rc = oo_gpu_rx_wait(p->gpu, c->ticket);
        c->busy = 0;
        if( rc < 0 )
          return rc;
      }
      gen = oo_gpu_rx_table_gen(p->gpu);
      i = (uint32_t)-1;  /* from the rest's first event */
      m = 0;
    }
  }
  *st = c->st;
  return 0;
}

int oo_rx_poll_evs(oo_rx_poll* p, const oo_rx_poll_ev* evs, uint32_t n,
                   oo_rx_poll_stats* stats)
{
  uint32_t done = 0, issued, k;
  int cur = 0, rc;
  if( p == NULL || stats == NULL || (n > 0 && evs == NULL) )
    return -EINVAL;
  if( n > (uint32_t)0x7fffffff )
    return -EINVAL;
  if( n == 0 )
    return 0;
  /* Chunk i+1 is submitted before chunk i is waited for, so its transform
   * overlaps chunk i's dispatch.  Each chunk's counters start from the
   * counters with every earlier chunk in (it completes after them). */
  k = n < p->cfg.evs_per_poll ? n : p->cfg.evs_per_poll;
  if( (rc = chunk_submit(p, &p->ch[0], evs, k, stats)) < 0 )
    return rc;
  issued = k;
  for( ;; ) {
    struct chunk* c = &p->ch[cur];
    struct chunk* nx = &p->ch[cur ^ 1];
    int sub_rc = 0, more = issued < n;
    uint64_t gen;
    oo_rx_poll_stats base;
    if( more ) {
      /* the next chunk's counters start where this one's will end: they
       * are rebased when this one completes */
      memset(&base, 0, sizeof(base));
      k = n - issued < p->cfg.evs_per_poll ? n - issued : p->cfg.evs_per_poll;
      sub_rc = chunk_submit(p, nx, evs + issued, k, &base);
    }
    const uint32_t cn = c->n;  /* (a re-transformed rest replaces c's events) */
    gen = oo_gpu_rx_table_gen(p->gpu);
    rc = chunk_complete(p, c, stats);
    if( rc == 0 && more && sub_rc == 0 && oo_gpu_rx_table_gen(p->gpu) != gen ) {
      /* This chunk's callbacks changed the tables (a filter inserted on an
       * accept, removed on a close, next to ci_netif_filter_insert / _remove)
       * after the next chunk was transformed: the reference loop, one event
       * after another, would run the next packets on the new tables.  The
       * next chunk is transformed again (its first transform's records are
       * discarded; nothing was dispatched from them). */
      if( nx->busy ) {
        (void)oo_gpu_rx_wait(p->gpu, nx->ticket);
        nx->busy = 0;
      }
      memset(&base, 0, sizeof(base));
      sub_rc = chunk_submit(p, nx, evs + issued, k, &base);
      ++nx->st.n_resubmit;
    }
    if( rc < 0 ) {
      if( more && sub_rc == 0 && nx->busy ) {  /* it must not outlive the call */
        (void)oo_gpu_rx_wait(p->gpu, nx->ticket);
        nx->busy = 0;
      }
      return done > 0 ? (int)done : rc;
    }
    done += cn;
    if( !more )
      return (int)done;
    if( sub_rc < 0 )
      return done > 0 ? (int)done : sub_rc;
    /* rebase the next chunk's counters on everything completed so far */
    {
      uint64_t* a = (uint64_t*)&nx->st;
      const uint64_t* s = (const uint64_t*)stats;
      size_t j;
      for( j = 0; j < sizeof(oo_rx_poll_stats) / sizeof(uint64_t); ++j )
        a[j] += s[j];
    }
    issued += k;
    cur ^= 1;
  }
}
