/* SPDX-License-Identifier: BSD-2-Clause */
/*
 * oo_rx_poll.c -- batched software-RX branch of ci_netif_poll_evq over
 * liboo_gpu_rx.  See include/oo_rx_poll.h for the contract; each step below
 * names the reference code whose behaviour it keeps.
 *
 * One call of oo_rx_poll_evs:
 *   1. classify each event (netif_event.c:1715-1742 RX branch, :1843
 *      discard_rx_multi_pkts): transform / release / other_ev, and count the
 *      per-event stats the loop keeps (rx_evs, rx_discard_*);
 *   2. pack the frames to transform into one registered host buffer at 64-B
 *      alignment and run oo_gpu_rx_batch over them (one device batch per
 *      evs_per_poll events);
 *   3. walk the records in event order and dispatch each one through the
 *      callback table, counting what the replaced code counts.
 */
#include "oo_rx_poll.h"

#include <errno.h>
#include <stdlib.h>
#include <string.h>

struct oo_rx_poll {
  oo_gpu_rx_ctx*   gpu;
  oo_rx_poll_cfg   cfg;
  oo_rx_poll_ops   ops;
  uint8_t*         pack;       /* packed frames of one batch (registered) */
  uint64_t         pack_bytes;
  oo_gpu_pkt_desc* desc;       /* evs_per_poll descriptors (registered)   */
  oo_gpu_rx_result* rec;       /* evs_per_poll records (registered)       */
  uint32_t*        ev_of;      /* batch slot -> event index               */
  uint8_t*         what;       /* per event of the batch: enum step       */
  int              registered; /* pack/desc/rec registered with the ctx   */
};

enum { W_TRANSFORM = 0, W_RELEASE = 1, W_OTHER = 2 };

static uint64_t up64(uint64_t x) { return (x + 63u) & ~(uint64_t)63u; }

static uint16_t be16_at(const uint8_t* p) { return (uint16_t)(p[0] << 8 | p[1]); }

static uint32_t be32_at(const uint8_t* p)
{
  return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}

static void* alloc64(uint64_t bytes)
{
  void* p = NULL;
  if( posix_memalign(&p, 4096, bytes ? bytes : 64) != 0 )
    return NULL;
  memset(p, 0, bytes ? bytes : 64);
  return p;
}

void oo_rx_poll_close(oo_rx_poll* p)
{
  if( p == NULL )
    return;
  if( p->registered ) {
    oo_gpu_rx_host_unregister(p->gpu, p->pack);
    oo_gpu_rx_host_unregister(p->gpu, p->desc);
    oo_gpu_rx_host_unregister(p->gpu, p->rec);
  }
  free(p->pack);
  free(p->desc);
  free(p->rec);
  free(p->ev_of);
  free(p->what);
  free(p);
}

int oo_rx_poll_open(oo_rx_poll** out, oo_gpu_rx_ctx* gpu, const oo_rx_poll_cfg* cfg,
                    const oo_rx_poll_ops* ops)
{
  oo_rx_poll* p;
  uint32_t n;
  if( out == NULL || gpu == NULL || cfg == NULL || ops == NULL )
    return -EINVAL;
  *out = NULL;
  n = cfg->evs_per_poll;
  if( n == 0 || n > OO_RX_POLL_MAX_EVS || cfg->buf_size == 0 ||
      (cfg->buf_size & (cfg->buf_size - 1)) != 0 || cfg->buf_size > 65536 ||
      (cfg->pkt_bufs == NULL && cfg->pkt_bufs_bytes != 0) )
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
  /* A frame never exceeds the 16-bit event length; within a buffer it
   * never exceeds buf_size. */
  p->pack_bytes = (uint64_t)n * up64(cfg->buf_size);
  p->pack = alloc64(p->pack_bytes);
  p->desc = alloc64(sizeof(oo_gpu_pkt_desc) * (uint64_t)n);
  p->rec = alloc64(sizeof(oo_gpu_rx_result) * (uint64_t)n);
  p->ev_of = malloc(sizeof(uint32_t) * (uint64_t)n);
  p->what = malloc(n);
  if( !p->pack || !p->desc || !p->rec || !p->ev_of || !p->what ) {
    oo_rx_poll_close(p);
    return -ENOMEM;
  }
  /* Registered staging: the H2D / D2H copies run straight from these
   * buffers (no second memcpy through the context's pinned slots). */
  if( oo_gpu_rx_host_register(gpu, p->pack, p->pack_bytes, NULL) == 0 ) {
    if( oo_gpu_rx_host_register(gpu, p->desc, sizeof(oo_gpu_pkt_desc) * (uint64_t)n,
                                NULL) == 0 ) {
      if( oo_gpu_rx_host_register(gpu, p->rec, sizeof(oo_gpu_rx_result) * (uint64_t)n,
                                  NULL) == 0 )
        p->registered = 1;
      else
        oo_gpu_rx_host_unregister(gpu, p->desc);
    }
    if( !p->registered )
      oo_gpu_rx_host_unregister(gpu, p->pack);
  }
  *out = p;
  return 0;
}

/* The frame of an event inside the pool, or NULL if it does not lie inside
 * it (such an event is not the shim's to take). */
static const uint8_t* frame_of(const oo_rx_poll* p, const oo_rx_poll_ev* e)
{
  uint64_t off = (uint64_t)e->rq_id * p->cfg.buf_size + e->ofs;
  if( e->ofs >= p->cfg.buf_size || off > p->cfg.pkt_bufs_bytes ||
      e->len > p->cfg.pkt_bufs_bytes - off )
    return NULL;
  return (const uint8_t*)p->cfg.pkt_bufs + off;
}

/* Step 1: what the poll loop does with an event before any transform
 * (netif_event.c:1715-1742 plain RX, :1131-1191 discard). */
static int classify(const oo_rx_poll* p, const oo_rx_poll_ev* e, oo_rx_poll_stats* st)
{
  const int whole = (e->flags & (OO_RX_EV_SOP | OO_RX_EV_CONT)) == OO_RX_EV_SOP;
  if( e->discard == 0 ) {
    ++st->rx_evs;                                          /* :1718 */
    if( !p->cfg.sw_verify || !whole || frame_of(p, e) == NULL )
      return W_OTHER;                                      /* reference branch */
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
    /* The future seam (see oo_rx_poll.h): TCP decided in stage 1, or UDP
     * unicast with a single match in its deciding stage. */
    if( r->reason == OO_RX_R_DELIVER )
      future = r->proto == 6 ? r->stage == 1
             : r->proto == 17 && !(r->flags & (OO_RX_F_MCAST | OO_RX_F_MULTI)) &&
               r->nmatch == 1;
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

static int run_batch(oo_rx_poll* p, const oo_rx_poll_ev* evs, uint32_t n,
                     oo_rx_poll_stats* st)
{
  uint32_t i, m = 0;
  uint64_t at = 0;
  oo_rx_poll_stats local;
  int rc;
  /* Counters land only if the batch does: on a device failure the caller
   * still owns every event from this batch on. */
  local = *st;
  for( i = 0; i < n; ++i ) {
    const oo_rx_poll_ev* e = &evs[i];
    p->what[i] = (uint8_t)classify(p, e, &local);
    if( p->what[i] == W_TRANSFORM ) {
      oo_gpu_pkt_desc* d = &p->desc[m];
      memcpy(p->pack + at, frame_of(p, e), e->len);
      d->frame_off = at;
      d->len = e->len;
      d->intf_i = e->intf_i;
      d->rsvd = 0;
      p->ev_of[m++] = i;
      at += up64(e->len);
    }
  }
  if( m > 0 ) {
    rc = oo_gpu_rx_batch(p->gpu, p->pack, at, p->desc, m, p->rec, NULL);
    if( rc < 0 )
      return rc;
    ++local.n_batches;
  }
  /* Step 3, in event order. */
  m = 0;
  for( i = 0; i < n; ++i ) {
    const oo_rx_poll_ev* e = &evs[i];
    if( p->what[i] == W_OTHER ) {
      ++local.n_other;
      p->ops.other_ev(p->ops.arg, e);
    }
    else if( p->what[i] == W_RELEASE ) {
      ++local.n_release;
      p->ops.release(p->ops.arg, e->rq_id, frame_of(p, e), NULL);
    }
    else {
      const oo_gpu_rx_result* r = &p->rec[m++];
      const uint8_t* frame = frame_of(p, e);
      if( r->reason >= OO_RX_R_DROP_BASE ) {
        count_drop(r, &local);
        ++local.n_release;
        p->ops.release(p->ops.arg, e->rq_id, frame, r);
      }
      else {
        if( e->discard ) {         /* the discard path's double count, :1189-1190 */
          ++local.rx_evs;
          ++local.rx_sw_csum_pass;
        }
        dispatch(p, e->rq_id, frame, r, &local);
      }
    }
  }
  *st = local;
  return 0;
}

int oo_rx_poll_evs(oo_rx_poll* p, const oo_rx_poll_ev* evs, uint32_t n,
                   oo_rx_poll_stats* stats)
{
  uint32_t done = 0;
  if( p == NULL || stats == NULL || (n > 0 && evs == NULL) )
    return -EINVAL;
  if( n > (uint32_t)0x7fffffff )
    return -EINVAL;
  while( done < n ) {
    uint32_t k = n - done < p->cfg.evs_per_poll ? n - done : p->cfg.evs_per_poll;
    int rc = run_batch(p, evs + done, k, stats);
    if( rc < 0 )
      return rc;
    done += k;
  }
  return (int)n;
}
