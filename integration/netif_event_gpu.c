/* SPDX-License-Identifier: BSD-2-Clause */
/*
 * netif_event_gpu.c -- CHECK-ONLY integration of the batched RX branch
 * (include/oo_rx_poll.h, src/shim/oo_rx_poll.c) into Onload's
 * ci_netif_poll_evq.  Not shipped and not built into anything: `make
 * check-integration` compiles it in this container against the reference's
 * own sources (it includes src/lib/transport/ip/netif_event.c, so every
 * static it calls -- handle_rx_pkt, the post-future helpers -- is the real
 * one, with the real signatures), which is what a maintainer applying
 * INTEGRATION.md §2 to the tree would compile.
 *
 * What it binds:
 *   post_future  -> ci_tcp_handle_rx_post_future (tcp_rx.h:198-214) with a
 *                   struct ci_tcp_rx_future built as ci_tcp_handle_rx_pre_future
 *                   would (tcp_rx.h:150-184: rxp.ni/pkt/tcp/seq/ack/hash,
 *                   pf.tcp_rx.pay_len), or ci_udp_handle_rx_post_future
 *                   (udp_internal.h:116-134) after the recvq / memory test
 *                   of ci_udp_rx_deliver_to_future (udp_internal.h:41-52)
 *   full_handler -> ci_tcp_handle_rx / ci_udp_handle_rx (what a NULL future
 *                   falls back to)
 *   pkt_handler  -> handle_rx_pkt (netif_event.c:250)
 *   release      -> ci_netif_pkt_release_rx_1ref
 *   other_ev     -> back to the existing per-event loop
 * and adds the shim's counters to the stack's (stats_def.h, ip_stats_ops.h).
 */
#include "netif_event.c"           /* -I src/lib/transport/ip */
#include "oo_rx_poll.h"            /* -I include (this repo)  */

struct gpu_poll_ctx {
  ci_netif* ni;
  struct ci_netif_poll_state* ps;
  const oo_rx_poll_ev* evs;        /* the shim's events of this call       */
  uint8_t* handback;               /* per shim event: other_ev gave it back */
};

static ci_ip_pkt_fmt* gpu_pkt(ci_netif* ni, uint32_t id)
{
  oo_pkt_p pp;
  OO_PP_INIT(ni, pp, id);
  return PKT_CHK(ni, pp);
}

/* What ci_parse_rx_vlan and handle_rx_csum_bad leave in the packet
 * (netif_event.c:116-132, :1024-1076). */
static void gpu_restore(ci_ip_pkt_fmt* pkt, const oo_gpu_rx_result* r, int frame_len)
{
  pkt->pay_len = frame_len;
  oo_offbuf_init(&pkt->buf, PKT_START(pkt), pkt->pay_len);
  pkt->pkt_eth_payload_off = pkt->pkt_start_off + ((r->flags & OO_RX_F_VLAN) ? 18 : 14);
  pkt->vlan = r->vlan;
  if( r->flags & OO_RX_F_IP6 )
    pkt->flags |= CI_PKT_FLAG_IS_IP6;
  else
    pkt->flags &= ~CI_PKT_FLAG_IS_IP6;
}

static int gpu_frame_len(const oo_gpu_rx_result* r, ci_ip_pkt_fmt* pkt)
{
  return pkt->pay_len;  /* set from the event before the batch */
}

static int gpu_post_future(void* arg, uint32_t id, const uint8_t* frame,
                           const oo_gpu_rx_result* r, const oo_rx_poll_future* f)
{
  struct gpu_poll_ctx* c = arg;
  ci_netif* ni = c->ni;
  ci_ip_pkt_fmt* pkt = gpu_pkt(ni, id);
  char* l4 = PKT_START(pkt) + f->l4_off;
  gpu_restore(pkt, r, gpu_frame_len(r, pkt));
  if( r->proto == IPPROTO_TCP ) {
    struct ci_tcp_rx_future fut;
    fut.socket = ID_TO_SOCK(ni, f->sock);
    fut.rxp.ni = ni;
    fut.rxp.pkt = pkt;
    fut.rxp.tcp = (ci_tcp_hdr*) l4;
    fut.rxp.seq = f->seq;
    fut.rxp.ack = f->ack;
    fut.rxp.hash = f->hash;
    pkt->pf.tcp_rx.pay_len = f->pay_len;
    ci_tcp_handle_rx_post_future(ni, c->ps, pkt, (ci_tcp_hdr*) l4, f->ip_paylen, &fut);
    return 0;
  }
  else {
    struct ci_udp_rx_future fut;
    ci_udp_state* us = SOCK_TO_UDP(ID_TO_SOCK(ni, f->sock));
    if( ci_udp_recv_q_pkts(&us->recv_q) >= us->stats.max_recvq_pkts ||
        (ni->state->mem_pressure & OO_MEM_PRESSURE_CRITICAL) )
      return 1;                    /* the NULL future: full handler */
    fut.socket = us;
    pkt->pf.udp.pay_len = f->pay_len;
    ci_udp_handle_rx_post_future(ni, pkt, (ci_udp_hdr*) l4, f->ip_paylen, &fut);
    return 0;
  }
}

static void gpu_full_handler(void* arg, uint32_t id, const uint8_t* frame,
                             const oo_gpu_rx_result* r)
{
  struct gpu_poll_ctx* c = arg;
  ci_ip_pkt_fmt* pkt = gpu_pkt(c->ni, id);
  char* l4 = PKT_START(pkt) + r->l4_off;
  gpu_restore(pkt, r, gpu_frame_len(r, pkt));
  if( r->proto == IPPROTO_TCP )
    ci_tcp_handle_rx(c->ni, c->ps, pkt, (ci_tcp_hdr*) l4, r->ip_paylen);
  else
    ci_udp_handle_rx(c->ni, pkt, (ci_udp_hdr*) l4, r->ip_paylen);
}

static void gpu_pkt_handler(void* arg, uint32_t id, const uint8_t* frame,
                            const oo_gpu_rx_result* r)
{
  struct gpu_poll_ctx* c = arg;
  ci_ip_pkt_fmt* pkt = gpu_pkt(c->ni, id);
  gpu_restore(pkt, r, gpu_frame_len(r, pkt));
  handle_rx_pkt(c->ni, c->ps, pkt);
}

static void gpu_release(void* arg, uint32_t id, const uint8_t* frame,
                        const oo_gpu_rx_result* r)
{
  struct gpu_poll_ctx* c = arg;
  ci_netif_pkt_release_rx_1ref(c->ni, gpu_pkt(c->ni, id));
}

static void gpu_other_ev(void* arg, const oo_rx_poll_ev* e)
{
  struct gpu_poll_ctx* c = arg;
  c->handback[e - c->evs] = 1;     /* the existing loop takes the original */
}

/* Discard subtypes as the shim's flags (the inverse of
 * ef_vi_receive_get_discard_type, ef_vi.h:1903-1921). */
static uint16_t gpu_discard_flags(unsigned subtype)
{
  switch( subtype ) {
  case EF_EVENT_RX_DISCARD_CSUM_BAD:  return OO_RX_DISCARD_L4_CSUM_ERR;
  case EF_EVENT_RX_DISCARD_CRC_BAD:   return OO_RX_DISCARD_ETH_FCS_ERR;
  case EF_EVENT_RX_DISCARD_TRUNC:     return OO_RX_DISCARD_ETH_LEN_ERR;
  default:                            return 0x10;  /* another class */
  }
}

static void gpu_add_stats(ci_netif* ni, const oo_rx_poll_stats* s)
{
  CITP_STATS_NETIF_ADD(ni, rx_evs, s->rx_evs);
  CITP_STATS_NETIF_ADD(ni, rx_sw_csum_pass, s->rx_sw_csum_pass);
  CITP_STATS_NETIF_ADD(ni, rx_discard_csum_bad, s->rx_discard_csum_bad);
  CITP_STATS_NETIF_ADD(ni, rx_discard_len_err, s->rx_discard_len_err);
  CITP_STATS_NETIF_ADD(ni, rx_discard_crc_bad, s->rx_discard_crc_bad);
  CITP_STATS_NETIF_ADD(ni, rx_discard_other, s->rx_discard_other);
  CITP_STATS_NETIF_ADD(ni, ip_options, s->ip_options);
#if CI_CFG_SUPPORT_STATS_COLLECTION
  ni->state->stats_snapshot.ip.in_recvs += s->in_recvs;
  ni->state->stats_snapshot.ip.in_hdr_errs += s->in_hdr_errs;
  ni->state->stats_snapshot.ip.in_delivers += s->in_delivers;
  ni->state->stats_snapshot.ip.in6_recvs += s->in6_recvs;
  ni->state->stats_snapshot.ip.in6_hdr_errs += s->in6_hdr_errs;
  ni->state->stats_snapshot.ip.in6_delivers += s->in6_delivers;
  ni->state->stats_snapshot.tcp.tcp_in_segs += s->tcp_in_segs;
  ni->state->stats_snapshot.udp.udp_in_dgrams += s->udp_in_dgrams;
  ni->state->stats_snapshot.udp.udp_in_errs += s->udp_in_errs;
#endif
}

/* Per-stack state: the device context, the shim and the callback context it
 * was opened with (ops.arg), refreshed for each batch, and the RX events
 * queued over one ci_netif_poll_evq pass (ci_netif_rx_gpu_queue): the
 * shim's view of each and the original, for the existing loop. */
struct ci_netif_gpu_rx {
  oo_gpu_rx_ctx* gpu;
  oo_rx_poll* poll;
  struct gpu_poll_ctx c;
  int cap, n;                      /* queued events, capacity               */
  oo_rx_poll_ev* q;
  ef_event* orig;
  uint8_t* handback;
};

void ci_netif_rx_gpu_close(struct ci_netif_gpu_rx* g);

/* At stack creation, next to ci_netif_filter_init (netif_init.c:105-108).
 * umem: the AF_XDP UMEM the RX ring's addresses index (chunk 2048,
 * tcp_helper_resource.c:2205-2208; efxdp_vi.c:337-348).  The shim reads
 * frames in place (the UMEM registered with the device) and leaves a pass
 * whose batch would cost more than the per-event loop to that loop
 * (OO_RX_POLL_CROSSOVER). */
int ci_netif_rx_gpu_open(ci_netif* ni, struct ci_netif_gpu_rx* g, int device,
                         const void* umem, uint64_t umem_bytes)
{
  oo_gpu_rx_cfg cfg;
  oo_rx_poll_cfg pcfg;
  oo_rx_poll_ops ops = { gpu_post_future, gpu_full_handler, gpu_pkt_handler,
                         gpu_release, gpu_other_ev, &g->c };
  int i, rc;
  memset(g, 0, sizeof(*g));
  /* A pass polls 16 events at a time until evs_per_poll (:1697, :1892). */
  g->cap = NI_OPTS(ni).evs_per_poll + 16;
  g->q = calloc(g->cap, sizeof(*g->q));
  g->orig = calloc(g->cap, sizeof(*g->orig));
  g->handback = calloc(g->cap, 1);
  if( g->q == NULL || g->orig == NULL || g->handback == NULL ) {
    ci_netif_rx_gpu_close(g);
    return -ENOMEM;
  }
  memset(&cfg, 0, sizeof(cfg));
  cfg.device = device;
  cfg.max_socks = ni->state->n_ep_bufs;
  cfg.ip4_table_log2 = ci_log2_ge(ni->filter_table->table_size_mask + 1, 16);
  cfg.ip6_table_log2 = ci_log2_ge(ni->ip6_filter_table->table_size_mask + 1, 1);
  cfg.n_intf = oo_stack_intf_max(ni);
  for( i = 0; i < cfg.n_intf; ++i )
    cfg.intf_hwport[i] = ni->state->intf_i_to_hwport[i];
  cfg.host_stage_bytes = (uint64_t) g->cap * 2048;
  cfg.host_stage_pkts = g->cap;
  if( (rc = oo_gpu_rx_open(&g->gpu, &cfg)) < 0 ) {
    g->gpu = NULL;
    ci_netif_rx_gpu_close(g);
    return rc;
  }
  memset(&pcfg, 0, sizeof(pcfg));
  pcfg.pkt_bufs = umem;
  pcfg.pkt_bufs_bytes = umem_bytes;
  pcfg.buf_size = 2048;
  pcfg.evs_per_poll = g->cap;
  pcfg.sw_verify = 1;              /* AF_XDP: no NIC checksum verdict */
  pcfg.flags = OO_RX_POLL_ZERO_COPY | OO_RX_POLL_CROSSOVER;
  g->c.ni = ni;
  if( (rc = oo_rx_poll_open(&g->poll, g->gpu, &pcfg, &ops)) < 0 ) {
    g->poll = NULL;
    ci_netif_rx_gpu_close(g);
  }
  return rc;
}

/* At stack teardown (and on ci_netif_rx_gpu_open's failure paths): the shim,
 * the device context and the pass's queue.  Idempotent. */
void ci_netif_rx_gpu_close(struct ci_netif_gpu_rx* g)
{
  if( g->poll != NULL )
    oo_rx_poll_close(g->poll);
  if( g->gpu != NULL )
    oo_gpu_rx_close(g->gpu);
  free(g->q);
  free(g->orig);
  free(g->handback);
  g->poll = NULL;
  g->gpu = NULL;
  g->q = NULL;
  g->orig = NULL;
  g->handback = NULL;
  g->cap = g->n = 0;
}

/* The shim's view of an RX / RX_DISCARD event (netif_event.c:1717-1736,
 * :1843): 1, or 0 for another event type. */
static int gpu_ev(ci_netif* ni, ef_vi* evq, int intf_i, const ef_event* ev,
                  oo_rx_poll_ev* e)
{
  oo_pkt_p pp;
  ci_ip_pkt_fmt* pkt;
  memset(e, 0, sizeof(*e));
  if( EF_EVENT_TYPE(*ev) == EF_EVENT_TYPE_RX ) {
    OO_PP_INIT(ni, pp, EF_EVENT_RX_RQ_ID(*ev));
    pkt = PKT_CHK(ni, pp);
    if( evq->nic_type.arch == EF_VI_ARCH_AF_XDP )   /* :1724-1727 */
      pkt->pkt_start_off = ev->rx.ofs - CI_MEMBER_OFFSET(ci_ip_pkt_fmt, dma_start);
    e->rq_id = EF_EVENT_RX_RQ_ID(*ev);
    e->len = EF_EVENT_RX_BYTES(*ev) - evq->rx_prefix_len;
    e->flags = ev->rx.flags;
  }
  else if( EF_EVENT_TYPE(*ev) == EF_EVENT_TYPE_RX_DISCARD ) {
    OO_PP_INIT(ni, pp, EF_EVENT_RX_DISCARD_RQ_ID(*ev));
    pkt = PKT_CHK(ni, pp);
    e->rq_id = EF_EVENT_RX_DISCARD_RQ_ID(*ev);
    e->len = EF_EVENT_RX_DISCARD_BYTES(*ev) - evq->rx_prefix_len;
    e->flags = ev->rx_discard.flags;
    e->discard = gpu_discard_flags(EF_EVENT_RX_DISCARD_TYPE(*ev));
  }
  else {
    return 0;
  }
  e->ofs = (uint16_t)(pkt->pkt_start_off + CI_MEMBER_OFFSET(ci_ip_pkt_fmt, dma_start));
  e->intf_i = (int16_t) intf_i;
  pkt->pay_len = e->len;
  return 1;
}

/* Inside ci_netif_poll_evq's do-loop, after each ef_eventq_poll (:1697): its
 * RX and RX_DISCARD events join the pass's queue; every other event -- and
 * any RX event the full queue cannot take -- is copied to other[] in order,
 * for the loop's existing switch now.  Returns how many. */
int ci_netif_rx_gpu_queue(ci_netif* ni, struct ci_netif_gpu_rx* g, ef_vi* evq,
                          int intf_i, const ef_event* ev, int n_evs, ef_event* other)
{
  int i, n_other = 0;
  for( i = 0; i < n_evs; ++i ) {
    if( g->n < g->cap && gpu_ev(ni, evq, intf_i, &ev[i], &g->q[g->n]) ) {
      g->orig[g->n] = ev[i];
      ++g->n;
    }
    else {
      other[n_other++] = ev[i];
    }
  }
  return n_other;
}

/* Once per pass, after the do-loop (before :1915): the queued events as one
 * batch.  Events the shim hands back (other_ev: not whole-buffer, outside
 * the pool, or a pass the crossover leaves to the loop) and -- if the
 * device fails -- every event it did not get to are copied to leftover[]
 * (capacity g->cap) in their original order, for the existing per-event
 * code.  Returns how many. */
int ci_netif_rx_gpu_flush(ci_netif* ni, struct ci_netif_poll_state* ps,
                          struct ci_netif_gpu_rx* g, ef_event* leftover)
{
  oo_rx_poll_stats st;
  int i, handled, n_left = 0;
  if( g->n == 0 )
    return 0;
  memset(&st, 0, sizeof(st));
  memset(g->handback, 0, (size_t) g->n);
  g->c.ps = ps;
  g->c.evs = g->q;
  g->c.handback = g->handback;
  /* n, or fewer if the device failed part-way: events from `handled` on ran
   * no callback and added no counter (oo_rx_poll.h) -- the CPU loop takes
   * them, so nothing is released or delivered twice. */
  handled = oo_rx_poll_evs(g->poll, g->q, (uint32_t) g->n, &st);
  if( handled < 0 )
    handled = 0;
  gpu_add_stats(ni, &st);
  for( i = 0; i < g->n; ++i )
    if( i >= handled || g->handback[i] )
      leftover[n_left++] = g->orig[i];
  g->n = 0;
  return n_left;
}

/* The one-call form for a loop left as it is: the events of one
 * ef_eventq_poll (any number of them: the queue is flushed whenever it
 * fills, nothing is dropped) in one batch.  other[] and leftover[] as above;
 * returns how many events went to leftover[] (the non-RX ones first, then
 * those the batch handed back). */
int ci_netif_rx_batch_gpu(ci_netif* ni, struct ci_netif_poll_state* ps,
                          struct ci_netif_gpu_rx* g, ef_vi* evq, int intf_i,
                          const ef_event* ev, int n_evs, ef_event* leftover)
{
  int done = 0, n_left = 0;
  while( done < n_evs ) {
    const int k = n_evs - done < g->cap - g->n ? n_evs - done : g->cap - g->n;
    n_left += ci_netif_rx_gpu_queue(ni, g, evq, intf_i, ev + done, k, leftover + n_left);
    done += k;
    n_left += ci_netif_rx_gpu_flush(ni, ps, g, leftover + n_left);
  }
  return n_left;
}
