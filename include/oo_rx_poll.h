/* SPDX-License-Identifier: BSD-2-Clause */
/*
 * oo_rx_poll.h -- the batched software-RX branch of ci_netif_poll_evq, as a C
 * shim over liboo_gpu_rx (src/shim/oo_rx_poll.c, built to
 * onload_amd/liboo_rx_poll.so).
 *
 * Today Onload runs the receive transform one event at a time, with a
 * one-packet lag (src/lib/transport/ip/netif_event.c:1709-1742 -> __handle_rx_pkt
 * -> handle_rx_pkt :250-451, or on the software-checksum path
 * discard_rx_multi_pkts :1131-1191 -> handle_rx_csum_bad :1014-1128).  The shim
 * takes the RX events of one poll (<= evs_per_poll, :1892), runs the whole
 * transform for all of them in one oo_gpu_rx_batch call, and then, per record,
 * does what the reference does after the transform:
 *
 *   dropped by the checks (reason >= OO_RX_R_DROP_BASE)
 *       -> ops->release                       ci_netif_pkt_release_rx_1ref
 *          (netif_event.c:1175-1183; the check's own counter is bumped:
 *           in_hdr_errs :1031/:1048/:1055, in6_hdr_errs :1069,
 *           udp_in_errs :1116)
 *   IPv4 not on the fast path (IP4_FRAG, IP4_OPTS_BAD)
 *       -> ops->pkt_handler                   handle_rx_pkt (:288-373: it
 *          passes the packet to the kernel and does its own counting)
 *   a resolved "future" socket: IPv4 TCP decided in lookup stage 1
 *   (ci_tcp_handle_rx_pre_future, tcp_rx.h:150-184), or IPv4 UDP whose two
 *   lookup stages together match exactly one socket
 *   (ci_udp_rx_deliver_to_future, udp_internal.h:41-103: a second match in
 *   either stage gives the future up; the record's nmatch and
 *   OO_RX_F_UDP_S2 say so)
 *       -> ops->post_future                   ci_{tcp,udp}_handle_rx_post_future
 *          (tcp_rx.h:198-214, udp_internal.h:116-134) with future->socket set;
 *          a non-zero return means the socket cannot take it now (recvq
 *          full, memory pressure: host state the device cannot see) and the
 *          packet goes to ops->full_handler instead, as a NULL future would
 *   everything else that was handled (TCP stages 2/3, NO_MATCH,
 *   TCP_SCATTERED, IPv6, multicast/broadcast or multi-match UDP)
 *       -> ops->full_handler                  ci_tcp_handle_rx (tcp_rx.c:4681)
 *          / ci_udp_handle_rx (udp_rx.c:236), the handler a NULL future
 *          falls back to
 *
 * and keeps the stack counters the replaced code keeps (struct
 * oo_rx_poll_stats: the stats_def.h / ip_stats_ops.h counters, by name).
 * RX events the transform does not take -- multi-buffer (scatter) events,
 * plain events when sw_verify is 0, frames not inside one buffer of the pool
 * -- go to ops->other_ev unchanged, for the caller's existing per-event
 * code, which also counts their rx_evs (netif_event.c:1718); discard events
 * outside the checksum class are released (:1175-1183).
 *
 * All calls happen on the caller's thread, under the stack lock, before
 * oo_rx_poll_evs returns, in event order.  (An integration that queues
 * other_ev events for its old loop, as integration/netif_event_gpu.c does,
 * runs them after the batch's transformed packets: on AF_XDP, the
 * north-star case, only non-whole-buffer events take that path, and AF_XDP
 * delivers single-buffer frames, efxdp_vi.c:343-348.)
 *
 * The batch path: the events are taken evs_per_poll at a time, two device
 * batches in flight (the next one's transform overlaps this one's
 * dispatch).  With OO_RX_POLL_ZERO_COPY the packet-buffer pool is
 * registered with the device at open and each frame is read where the NIC
 * put it (over PCIe, no host copy); otherwise the frames of a batch are
 * gathered into a registered buffer first.  In place, the buffer bytes per
 * packet say nothing of the frames, so each batch sets the context's
 * mean-frame-length hint (oo_gpu_rx_set_len_hint) to the batch's mean for
 * its launch and clears it after: a context shared with other callers
 * should not rely on a hint of its own while a zero-copy poll runs.
 */
#ifndef OO_RX_POLL_H
#define OO_RX_POLL_H

#include <stdint.h>

#include "oo_gpu_rx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Largest evs_per_poll (CI_CFG_EVS_PER_POLL_MAX-sized batches are far
 * smaller; a poll of many rings at once may gather more). */
#define OO_RX_POLL_MAX_EVS 65536

/* ef_event.rx.flags bits the shim reads (ef_vi.h:335-337). */
#define OO_RX_EV_SOP  0x1u   /* EF_EVENT_FLAG_SOP  */
#define OO_RX_EV_CONT 0x2u   /* EF_EVENT_FLAG_CONT */

/* Discard-event flags (EF_VI_DISCARD_RX_*, ef_vi.h:629-660), as
 * discard_rx_multi_pkts receives them (netif_event.c:1131-1191). */
#define OO_RX_DISCARD_L4_CSUM_ERR    0x001u
#define OO_RX_DISCARD_L3_CSUM_ERR    0x002u
#define OO_RX_DISCARD_ETH_FCS_ERR    0x004u
#define OO_RX_DISCARD_ETH_LEN_ERR    0x008u
#define OO_RX_DISCARD_L3_CLASS_OTHER 0x100u

/* One RX (or RX_DISCARD) event as the poll loop sees it after
 * ef_eventq_poll: EF_EVENT_RX_RQ_ID, the frame offset in the buffer (AF_XDP
 * ev.rx.ofs, efxdp_vi.c:346-348) and EF_EVENT_RX_BYTES - rx_prefix_len.
 * 16 bytes. */
typedef struct oo_rx_poll_ev {
  uint32_t rq_id;     /* packet buffer id                                     */
  uint16_t ofs;       /* frame's first byte inside the buffer                 */
  uint16_t len;       /* frame length                                         */
  uint16_t flags;     /* OO_RX_EV_*                                           */
  uint16_t discard;   /* 0 = RX event, else OO_RX_DISCARD_* of a discard event */
  int16_t  intf_i;    /* pkt->intf_i                                          */
  uint16_t rsvd;
} oo_rx_poll_ev;

/* What the post-future helpers consume, read from the record and the frame:
 * struct ci_tcp_rx_future {socket, rxp.{hash, seq, ack}} (tcp_rx.h:136-139,
 * filled at :162-179) / struct ci_udp_rx_future {socket}
 * (udp_internal.h:27-29), plus the payload pointer and ip_paylen arguments
 * (netif_event.c:836-840). */
typedef struct oo_rx_poll_future {
  int32_t  sock;        /* future->socket (OO_SP)                             */
  uint32_t hash;        /* TCP: rxp.hash (stage-1 __onload_hash3)             */
  uint32_t seq;         /* TCP: rxp.seq = CI_BSWAP_BE32(tcp_seq_be32)         */
  uint32_t ack;         /* TCP: rxp.ack                                       */
  uint32_t pay_len;     /* UDP: pkt->pf.udp.pay_len (udp_len - 8);
                           TCP: pkt->pf.tcp_rx.pay_len (= ip_paylen)          */
  uint16_t l4_off;      /* payload = frame + l4_off (the TCP / UDP header)    */
  uint16_t ip_paylen;   /* post_future's ip_paylen argument                   */
} oo_rx_poll_future;

/* The per-stack counters the replaced code keeps, named as in
 * src/include/ci/internal/stats_def.h (netif stats) and ip_stats_ops.h
 * (ipv4 / ip6 / tcp / udp).  oo_rx_poll_evs adds to them. */
typedef struct oo_rx_poll_stats {
  uint64_t rx_evs;                  /* stats_def.h:57, netif_event.c:1718/:1189
                                       (events handed to other_ev excluded)    */
  uint64_t rx_sw_csum_pass;         /* stats_def.h:881, netif_event.c:1190      */
  uint64_t rx_discard_csum_bad;     /* stats_def.h:521, netif_event.c:1170      */
  uint64_t rx_discard_len_err;      /* netif_event.c:1165                        */
  uint64_t rx_discard_crc_bad;      /* netif_event.c:1167                        */
  uint64_t rx_discard_other;        /* netif_event.c:1172                        */
  uint64_t ip_options;              /* netif_event.c:181 (options parsed OK)     */
  uint64_t in_recvs;                /* ipv4, netif_event.c:282                   */
  uint64_t in_hdr_errs;             /* ipv4, netif_event.c:1031/1048/1055        */
  uint64_t in_delivers;             /* ipv4, netif_event.c:327/332               */
  uint64_t in6_recvs;               /* ip6,  netif_event.c:384                   */
  uint64_t in6_hdr_errs;            /* ip6,  netif_event.c:1069                  */
  uint64_t in6_delivers;            /* ip6,  netif_event.c:394/400               */
  uint64_t tcp_in_segs;             /* tcp_rx.h:182 (future), tcp_rx.c:4692      */
  uint64_t udp_in_dgrams;           /* udp_internal.h:101 (future), udp_rx.c:262 */
  uint64_t udp_in_errs;             /* netif_event.c:1116                        */
  /* shim's own dispatch tallies (not Onload stats) */
  uint64_t n_future;                /* post_future accepted                      */
  uint64_t n_future_declined;       /* post_future returned non-zero             */
  uint64_t n_full;                  /* full_handler calls                        */
  uint64_t n_pkt_handler;           /* pkt_handler calls                         */
  uint64_t n_release;               /* release calls                             */
  uint64_t n_other;                 /* other_ev calls                            */
  uint64_t n_batches;               /* oo_gpu_rx_batch calls                     */
  uint64_t n_resubmit;              /* chunks transformed again: a callback of the
                                       chunk before changed the tables           */
  uint64_t n_handback;              /* events of chunks left to the caller's
                                       per-event path (OO_RX_POLL_CROSSOVER)     */
} oo_rx_poll_stats;

/* The callback table: the integration maps these onto the stack's functions
 * (tests/c/ drive it with a recording table).  `id` is
 * the event's rq_id, `frame` the frame's first byte in the caller's pool. */
typedef struct oo_rx_poll_ops {
  int  (*post_future)(void* arg, uint32_t id, const uint8_t* frame,
                      const oo_gpu_rx_result* r, const oo_rx_poll_future* f);
  void (*full_handler)(void* arg, uint32_t id, const uint8_t* frame,
                       const oo_gpu_rx_result* r);
  void (*pkt_handler)(void* arg, uint32_t id, const uint8_t* frame,
                      const oo_gpu_rx_result* r);
  void (*release)(void* arg, uint32_t id, const uint8_t* frame,
                  const oo_gpu_rx_result* r);
  void (*other_ev)(void* arg, const oo_rx_poll_ev* ev);
  void* arg;
} oo_rx_poll_ops;

typedef struct oo_rx_poll_cfg {
  const void* pkt_bufs;     /* packet-buffer pool / UMEM base (host memory)   */
  uint64_t    pkt_bufs_bytes;
  uint32_t    buf_size;     /* bytes per buffer (AF_XDP chunk: 2048, a power of
                               two; tcp_helper_resource.c:2205-2208)          */
  uint32_t    evs_per_poll; /* events per batch, 1..OO_RX_POLL_MAX_EVS        */
  uint32_t    sw_verify;    /* 1: plain RX events take the software checksum
                               path too (no NIC checksum offload: AF_XDP, the
                               north-star case); 0: only discard events in the
                               checksum class do (:1155-1162), plain RX events
                               go to other_ev                                  */
  uint32_t    flags;        /* OO_RX_POLL_ZERO_COPY | OO_RX_POLL_CROSSOVER      */
  /* The cost model OO_RX_POLL_CROSSOVER uses (0: the default of each, the
   * values tools/poll_bench measured).  Per chunk of m frames
   * and B frame bytes the device batch costs
   *   gpu_fixed_ns + m gpu_pkt_ps + B gpu_byte_ps
   * and the caller's own per-event path (handle_rx_csum_bad one event at a
   * time) m cpu_pkt_ps + B cpu_byte_ps. */
  uint32_t    cpu_pkt_ps;   /* the per-event CPU path: ps per frame           */
  uint32_t    cpu_byte_ps;  /*   and per frame byte                           */
  uint32_t    gpu_fixed_ns; /* the device batch: fixed ns per chunk           */
  uint32_t    gpu_pkt_ps;   /*   ps per frame                                 */
  uint32_t    gpu_byte_ps;  /*   ps per frame byte (gather: the host copy too) */
} oo_rx_poll_cfg;

/* cfg.flags: register pkt_bufs with the device and read frames in place
 * (falls back to gathering if the pool cannot be registered -- it must be
 * whole pages no other registration holds, oo_gpu_rx_host_register; see
 * oo_rx_poll_zero_copy).  The shim unregisters it at oo_rx_poll_close, which
 * must come before the context's close and before the pool is unmapped. */
#define OO_RX_POLL_ZERO_COPY 0x1u
/* cfg.flags: a chunk whose device batch would cost more than the caller's
 * own per-event path (the cost model above) is not transformed: all its
 * events go to ops->other_ev unchanged and uncounted, exactly as if the
 * shim were not there, so the caller's loop runs them one at a time
 * (netif_event.c:1709-1742 / :1131-1191).  The branch is then never slower
 * than the loop it replaces, by the model. */
#define OO_RX_POLL_CROSSOVER 0x2u

typedef struct oo_rx_poll oo_rx_poll;

/* gpu: an open context with host staging (oo_gpu_rx_cfg.host_stage_*) large
 * enough for evs_per_poll frames of the largest size.  0 or -errno. */
int  oo_rx_poll_open(oo_rx_poll** out, oo_gpu_rx_ctx* gpu, const oo_rx_poll_cfg* cfg,
                     const oo_rx_poll_ops* ops);
void oo_rx_poll_close(oo_rx_poll* p);

/* Handle n events (any number: they are taken evs_per_poll at a time) and
 * add to *stats.  Returns n.  If the device fails, the call stops at the
 * failed batch: no callback has run and no counter was added for its events
 * and the later ones, which the caller still owns (the reference CPU path
 * can take them); the return value is then the number of events handled
 * before it (< n), or -errno if that is 0.  -EINVAL for bad arguments. */
int  oo_rx_poll_evs(oo_rx_poll* p, const oo_rx_poll_ev* evs, uint32_t n,
                    oo_rx_poll_stats* stats);

/* 1 if frames are read in place (OO_RX_POLL_ZERO_COPY took), 0 if they are
 * gathered, -EINVAL. */
int  oo_rx_poll_zero_copy(const oo_rx_poll* p);

#ifdef __cplusplus
}
#endif

#endif /* OO_RX_POLL_H */
