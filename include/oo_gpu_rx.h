/* SPDX-License-Identifier: BSD-2-Clause */
/*
 * oo_gpu_rx.h -- C ABI of the MI355X (gfx950) receive-path transform library.
 *
 * The library runs Onload's per-packet software receive transform on a batch
 * of frames held in GPU memory (HBM):
 *
 *   software checksum verify  handle_rx_csum_bad   src/lib/transport/ip/netif_event.c:1014-1128
 *     IPv4 header csum         ci_ip_csum_correct   netif_event.c:80-94
 *     TCP csum                 ci_tcp_csum_correct  netif_event.c:97-113
 *     UDP csum                 ci_udp_csum_correct  src/lib/transport/ip/udp_rx.c:101-121
 *   header parse               ci_parse_rx_vlan     netif_event.c:116-132
 *                              handle_rx_pkt        netif_event.c:250-451
 *                              ci_ip_options_parse  netif_event.c:135-185
 *   4-tuple socket demux       ci_udp_handle_rx     udp_rx.c:236-307 (2 stages)
 *                              ci_tcp_handle_rx     src/lib/transport/ip/tcp_rx.c:4681-4836 (3 stages)
 *                              ci_netif_filter_for_each_match      netif_table.c:234-319
 *                              ci_netif_filter_for_each_match_ip6  netif_table_ip6.c:110-189
 *
 * and returns one fixed 32-byte record per frame (the batched equivalent of the
 * pre-resolved "future" the RX poll loop already understands,
 * src/lib/transport/ip/udp_internal.h:27-134, tcp_rx.h:136-214).
 *
 * Conventions (same as the reference):
 *  - addresses and ports are network-order values held in host integers
 *    ("BE values in host integers"), exactly what a little-endian load of the
 *    wire bytes yields;
 *  - 0 or a positive count on success, -errno on failure (ef_vi style);
 *    per-packet outcomes are reason codes, never errors;
 *  - every pointer is plain memory owned by the caller unless stated; device
 *    pointers are HIP device addresses; `stream` is a hipStream_t passed as
 *    void* (NULL = the null stream).
 *
 * Threading: a context belongs to one Onload stack and is used by the holder
 * of that stack's lock (netif_event.c:1919).  Table updates and batches are
 * serialised at that lock, like oof's deferred filter ops
 * (src/lib/efthrm/oof_interface.c:184-217).
 */
#ifndef OO_GPU_RX_H
#define OO_GPU_RX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OO_GPU_RX_ABI_VERSION 5

/* intf_i -> hwport map size (CI_CFG_MAX_INTERFACES = 30,
 * src/include/ci/internal/transport_config_opt.h:29). */
#define OO_GPU_RX_MAX_INTF 32

/* ---------------------------------------------------------------------
 * Per-packet outcome (reason) codes, in the reference's check order.
 * reason < OO_RX_R_DROP_BASE  => handle_rx_csum_bad() returned 1 (handled)
 * reason >= OO_RX_R_DROP_BASE => it returned 0: the caller releases the pkt
 * --------------------------------------------------------------------- */
enum {
  OO_RX_R_DELIVER        = 0,  /* socket matched: sock/stage/nmatch valid      */
  OO_RX_R_NO_MATCH       = 1,  /* udp_rx.c:315-347 / tcp_rx.c:4838-4853       */
  OO_RX_R_IP4_FRAG       = 2,  /* MF/offset set: netif_event.c:293-295, :339   */
  OO_RX_R_IP4_OPTS_BAD   = 3,  /* ci_ip_options_parse error: :302-303          */
  OO_RX_R_TCP_SCATTERED  = 4,  /* frag_off not in {0,DF}: tcp_rx.c:4696-4699   */
  OO_RX_R_DROP_BASE      = 16,
  OO_RX_R_SHORT_L2       = 16, /* netif_event.c:1030                            */
  OO_RX_R_NOT_IP         = 17, /* :1078                                         */
  OO_RX_R_IP4_LEN        = 18, /* :1047                                         */
  OO_RX_R_IP4_CSUM       = 19, /* :1054                                         */
  OO_RX_R_IP6_LEN        = 20, /* :1067                                         */
  OO_RX_R_PROTO_OTHER    = 21, /* :1121                                         */
  OO_RX_R_TCP_SHORT      = 22, /* :1087                                         */
  OO_RX_R_TCP_CSUM       = 23, /* :1091 (incl. doff<5, hlen>ip_paylen)          */
  OO_RX_R_UDP_SHORT      = 24, /* :1106                                         */
  OO_RX_R_UDP_CSUM       = 25, /* :1110 (incl. udp_len<8 or >paylen; v6 csum 0) */
  OO_RX_R_COUNT          = 32
};

/* Record flags. */
#define OO_RX_F_IP6     0x01u  /* CI_PKT_FLAG_IS_IP6 (ip_shared_types.h:387)     */
#define OO_RX_F_VLAN    0x02u  /* 802.1Q tag parsed (netif_event.c:126-130)       */
#define OO_RX_F_CSUM_OK 0x04u  /* L3+L4 software checksum verified                */
#define OO_RX_F_MCAST   0x08u  /* daddr multicast/broadcast: host must keep
                                  delivering to every match (udp_rx.c:148-203)     */
#define OO_RX_F_MULTI   0x10u  /* nmatch > 1 in the deciding stage (UDP only)    */
#define OO_RX_F_TSO     0x20u  /* TCP header in the timestamp-option fast layout
                                  (doff 8, options NOP NOP TS 10: tcp_rx.c:4537-4543,
                                  CI_TCP_TSO_WORD ip_shared_types.h:2742); the host
                                  reads TSval/TSecr at l4_off + 24 / + 28         */
#define OO_RX_F_UDP_S2  0x40u  /* UDP decided in stage 1 with one match, and the
                                  stage-2 (laddr, lport) lookup matches too: the
                                  union the future rule counts holds more than one
                                  socket (udp_internal.h:41-52, :86-97)           */

/* One frame in the batch.  16 bytes. */
typedef struct oo_gpu_pkt_desc {
  uint64_t frame_off;   /* byte offset of the frame's first L2 byte in the
                           frame buffer (AF_XDP: addr - headroom,
                           efxdp_vi.c:326-352, netif_event.c:1724-1727)      */
  uint16_t len;         /* frame length in bytes (no FCS; ef_event.rx.len)  */
  int16_t  intf_i;      /* Onload interface index (pkt->intf_i)              */
  uint32_t rsvd;        /* must be 0                                          */
} oo_gpu_pkt_desc;

/* Per-frame result.  32 bytes, written for every descriptor.
 *
 * Fields are defined in stages; anything a stage does not reach is 0 (sock
 * is -1 unless reason == OO_RX_R_DELIVER):
 *  - always:                      reason, flags&VLAN, vlan
 *  - ether_type IPv4/IPv6 and
 *    frame >= pre_l3 + 20:        flags&IP6, proto, ip_paylen (low 16 bits of
 *                                 the int the reference computes)
 *  - handled (reason < 16):       flags&CSUM_OK, l4_off, ports, saddr, daddr
 *  - lookups ran (DELIVER or
 *    NO_MATCH):                   hash3 (stage-1 __onload_hash3, rxp.hash),
 *                                 flags&MCAST
 *  - DELIVER:                     sock, stage, nmatch, flags&MULTI,
 *                                 flags&UDP_S2 (IPv4 UDP, stage 1, nmatch 1)
 * For IPv6, saddr/daddr hold onload_addr_xor() of the address (the value the
 * hash consumes, src/include/onload/hash.h:31-42); the full addresses are in
 * the frame at l4_off - 32 and l4_off - 16.
 */
typedef struct oo_gpu_rx_result {
  uint8_t  reason;      /* OO_RX_R_*                                         */
  uint8_t  flags;       /* OO_RX_F_*                                         */
  uint8_t  stage;       /* 1..3 = deciding lookup stage, 0 = none            */
  uint8_t  proto;       /* IP protocol / IPv6 next header                    */
  uint16_t vlan;        /* pkt->vlan (12-bit VID)                            */
  uint16_t l4_off;      /* L4 header offset from the frame start             */
  uint16_t ip_paylen;   /* IPv4 tot_len-4*IHL / IPv6 payload_len             */
  uint16_t sport_be;    /* L4 source port, network order in host integer     */
  uint16_t dport_be;    /* L4 dest port                                      */
  uint16_t nmatch;      /* matching filter entries in the deciding stage;
                           TCP: 1 (its walk ends at the first match)         */
  uint32_t saddr_be;    /* IPv4 saddr / IPv6 addr xor-fold                   */
  uint32_t daddr_be;    /* IPv4 daddr / IPv6 addr xor-fold                   */
  int32_t  sock;        /* matched socket id (OO_SP) or -1                   */
  uint32_t hash3;       /* stage-1 __onload_hash3 (tcp rxp.hash)             */
} oo_gpu_rx_result;

/* Per-reason packet counts for one batch; the host maps them onto Onload's
 * stats (rx_discard_csum_bad stats_def.h:521, rx_discard_ip_options_bad :537,
 * udp_rx_no_match_drops :631, rx_sw_csum_pass :881, ...). */
typedef struct oo_gpu_rx_counters {
  uint32_t by_reason[OO_RX_R_COUNT];
} oo_gpu_rx_counters;

/* Socket-side fields the demux reads (netif_table.c:192-231,
 * netif_table_ip6.c:146-170; accessors src/include/ci/internal/ip.h:1315-1340).
 * Values are exactly what the reference accessors return for the socket. */
#define OO_GPU_RX_SOCK_CONNECTED 0x1u  /* CI_SOCK_FLAG_CONNECTED             */
#define OO_GPU_RX_SOCK_BIND2DEV  0x2u  /* rx_bind2dev_ifindex != CI_IFID_BAD */
typedef struct oo_gpu_rx_sock {
  uint32_t raddr_be32;        /* sock_raddr_be32(s)                          */
  uint16_t rport_be16;        /* sock_rport_be16(s)                          */
  uint16_t lport_be16;        /* sock_lport_be16(s)                          */
  uint8_t  protocol;          /* sock_protocol(s)                            */
  uint8_t  rsvd0;
  uint16_t flags;             /* OO_GPU_RX_SOCK_*                            */
  int16_t  bind2dev_vlan;     /* s->rx_bind2dev_vlan                         */
  uint16_t rsvd1;
  uint64_t bind2dev_hwports;  /* s->rx_bind2dev_hwports                      */
  uint8_t  raddr6[16];        /* sock_ip6_raddr(s)                           */
  uint8_t  rsvd2[8];
} oo_gpu_rx_sock;             /* 48 bytes                                     */

typedef struct oo_gpu_rx_cfg {
  int32_t  device;            /* HIP device ordinal; < 0 = host-only context
                                 (tables without a GPU; batch calls return
                                 -ENODEV)                                      */
  uint32_t max_socks;         /* socket ids are 0..max_socks-1 (EP buffers)  */
  uint8_t  ip4_table_log2;    /* >= 16 (netif_table.c:280 LPRP), <= 24;
                                 default 16 (ip.h:1790-1804)                  */
  uint8_t  ip6_table_log2;    /* 1..24; default 14 (netif_init.c:107-108)    */
  uint8_t  n_intf;            /* entries used in intf_hwport                 */
  uint8_t  rsvd;
  uint8_t  intf_hwport[OO_GPU_RX_MAX_INTF]; /* ni->state->intf_i_to_hwport   */
  uint64_t host_stage_bytes;  /* frame bytes per submit slot (0 = no host path) */
  uint32_t host_stage_pkts;   /* packets per submit slot                      */
  uint32_t rsvd2;
} oo_gpu_rx_cfg;

typedef struct oo_gpu_rx_ctx oo_gpu_rx_ctx;

/* Library / context lifetime.  close: 0, or -EBUSY while host memory is
 * still registered with the context (oo_gpu_rx_host_register): the context
 * stays open; the caller unregisters that memory -- before it unmaps or
 * frees it -- and closes again.  NULL: 0. */
int oo_gpu_rx_abi_version(void);
int oo_gpu_rx_open(oo_gpu_rx_ctx** ctx_out, const oo_gpu_rx_cfg* cfg);
int oo_gpu_rx_close(oo_gpu_rx_ctx* ctx);

/* Filter tables.  Replaces ci_netif_filter_insert / _remove
 * (netif_table.c:436-503 -> ci_ip4_netif_filter_insert :323-406,
 * ci_ip4_netif_filter_remove :447-495; IPv6 netif_table_ip6.c:192-345) for one
 * address family (af = 4 or 6).  Slot placement, route counts and tombstones
 * are identical to the reference.  laddr/raddr point at 4 (af 4) or 16 (af 6)
 * network-order bytes; raddr NULL means the wildcard.
 * insert: 0, -ENOBUFS (table full, :375), -EINVAL.  remove: 0 (also when the
 * filter is absent, :476-481), -EINVAL.
 * The result is decided at once on a host mirror; the change itself (and a
 * socket change, oo_gpu_rx_sock_set) is queued and applied to the HBM tables
 * by a device kernel on the stream of the next batch (or sync_tables), in
 * call order -- oof's deferred-op model (oof_interface.c:184-217).  Batches
 * already enqueued on any stream of the context finish before the change
 * lands; batches enqueued after it see it, on whatever stream.  No call
 * synchronises with the device for it. */
int oo_gpu_rx_table_insert(oo_gpu_rx_ctx* ctx, int af,
                           const void* laddr, uint16_t lport_be16,
                           const void* raddr, uint16_t rport_be16,
                           uint8_t protocol, int32_t sock_id);
int oo_gpu_rx_table_remove(oo_gpu_rx_ctx* ctx, int af,
                           const void* laddr, uint16_t lport_be16,
                           const void* raddr, uint16_t rport_be16,
                           uint8_t protocol, int32_t sock_id);
/* Exact-tuple slot lookup, ci_ip4_netif_filter_lookup (netif_table.c:86-143) /
 * ci_ip6_netif_filter_lookup (netif_table_ip6.c:13-66): slot index >= 0,
 * -ENOENT or -ELOOP. */
int oo_gpu_rx_table_lookup(oo_gpu_rx_ctx* ctx, int af,
                           const void* laddr, uint16_t lport_be16,
                           const void* raddr, uint16_t rport_be16,
                           uint8_t protocol);
/* Raw view of one table slot for diagnostics/tests: id_state (v4: id|state<<30,
 * v6: id with -1 tombstone / -2 empty), route_count, lport (v4 ext). */
int oo_gpu_rx_table_slot(oo_gpu_rx_ctx* ctx, int af, uint32_t slot,
                         uint32_t* id_state, int32_t* route_count,
                         uint16_t* lport_be16);
int oo_gpu_rx_sock_set(oo_gpu_rx_ctx* ctx, int32_t sock_id,
                       const oo_gpu_rx_sock* sock);
/* Apply pending table/socket changes to the device on `stream` now. */
int oo_gpu_rx_sync_tables(oo_gpu_rx_ctx* ctx, void* stream);
/* The number of table and socket changes made on the context so far
 * (insert, remove, sock_set, import): a caller that has batches in flight
 * compares it across its own callbacks to learn whether a batch submitted
 * before them was transformed on tables that have since changed. */
uint64_t oo_gpu_rx_table_gen(const oo_gpu_rx_ctx* ctx);
/* Which kernels transformed the context's last batch: 1 rx_kernel with the
 * 4-slot ring, 2 its 2-slot instance, 3 the split transform (win_kernel +
 * body_kernel with lockstep slots), 4 the split transform with the
 * per-group-sequence body_kernel, 5 the poll instance (12-slot ring, 8-packet
 * tiles: batches of at most 256 packets; a submit_mapped batch's completion
 * written by the kernel); 0 none yet.  For measurements: which kernels a
 * timed launch's duration covers. */
uint32_t oo_gpu_rx_last_path(const oo_gpu_rx_ctx* ctx);
/* Table maintenance so far: flushes of queued changes to the device, and how
 * the key index followed each -- rebuilt from the tables, or updated for the
 * flushed ops' keys alone (a flush of at most 1024 filter ops with no
 * socket change) -- and whether it answers lookups now (waits for the
 * device).  For tests and measurements. */
typedef struct oo_gpu_rx_table_stats {
  uint64_t flushes;
  uint64_t index_rebuilds;
  uint64_t index_updates;
  uint32_t index_on;
  uint32_t rsvd;
} oo_gpu_rx_table_stats;
int oo_gpu_rx_get_table_stats(oo_gpu_rx_ctx* ctx, oo_gpu_rx_table_stats* out);
/* Streams.  The context remembers the streams it launched on (nothing is
 * recorded per batch): a table change enqueues an event on each of them at
 * that moment and waits for it, so every stream used with the context must
 * stay valid until the context is closed -- or until this call, made before
 * destroying it, which records the stream's last event and stops using the
 * stream itself.  0 (also for a stream the context never used), -EIO. */
int oo_gpu_rx_stream_done(oo_gpu_rx_ctx* ctx, void* stream);

/* Table image: the context's whole table state (slot records with route
 * counts, tombstones and the socket fields they name; socket records) as one
 * flat blob, for replicating one stack's tables onto other GPUs (SURVEY.md
 * §8(e): broadcast once, then the same ops on every rank).  Layout: a 64-B
 * header {u32 magic "OOTB", u32 version, u32 ip4_log2, u32 ip6_log2,
 * u32 max_socks, u32 rsvd, u64 off_slot4, off_rc4, off_slot6, off_socks,
 * total}, then 32-B IPv4 slot records, i32 route counts, 64-B IPv6 slot
 * records, 48-B oo_gpu_rx_sock records.  Identical bytes from a host-only
 * context and a device context holding the same tables.
 * export: pending changes are applied first, then the image is copied to dst
 * (device or host memory; host memory for a host-only context) on `stream`,
 * asynchronously.  import: replaces the tables (pending changes dropped) from
 * src on `stream`; returns once the mirror is loaded.  Sizes must match the
 * context's: -EINVAL otherwise. */
uint64_t oo_gpu_rx_table_image_bytes(const oo_gpu_rx_ctx* ctx);
int oo_gpu_rx_table_export(oo_gpu_rx_ctx* ctx, void* dst, uint64_t bytes, void* stream);
int oo_gpu_rx_table_import(oo_gpu_rx_ctx* ctx, const void* src, uint64_t bytes,
                           void* stream);

/* The mean frame length of the batches to come, in bytes (0, the default:
 * infer it from the frame buffer's bytes per packet, right for packed
 * batches but not for an AF_XDP UMEM of 2048-B chunks).  The transform
 * compiles two instances of its kernel -- for frames under 1 KiB one that
 * keeps more waves per CU, since short frames are bound by the per-packet
 * header and lookup chain rather than the byte stream -- and
 * picks one per batch by this.  Results are identical either way.
 * 0 or -EINVAL. */
int oo_gpu_rx_set_len_hint(oo_gpu_rx_ctx* ctx, uint32_t mean_frame_len);

/* Launch settings, for measurements: which kernels transform a batch and
 * how its work is cut.  Results are identical under every setting; the
 * defaults (all fields 0, gshift -1; or t = NULL) are what DESIGN.md §2
 * measured fastest.  The library reads no environment: a deployment gets
 * exactly these defaults unless it calls this.  0 or -EINVAL. */
typedef struct oo_gpu_rx_tuning {
  uint32_t path;           /* 0 auto (frames within
                              the 128-B header window, 2^20+ packets: 3;
                              mixed sizes with long frames, 2^16+: 3; else 2
                              for under 1 KiB of buffer per packet, 1
                              otherwise);
                              1 one rx_kernel launch, 4-slot body ring;
                              2 the same with the 2-slot ring; 3 the split
                              transform (win_kernel + body_kernel); 4 the
                              poll instance (12-slot ring; a submit_mapped
                              batch's completion written by the kernel)    */
  uint32_t grid_pct;       /* % of the resident grid to launch (0: 100)       */
  uint32_t groups;         /* tile-claim groups at most (0: by frame size)    */
  int32_t  gshift;         /* a group's wave runs, log2 (-1: by frame size)   */
  uint32_t static_tiles;   /* 1: a static tile partition, no claims           */
  uint32_t tail_tile;      /* packets per tile at the batch's end (0: 32)     */
  uint32_t tail_per_wave;  /* such tiles per wave (0: 1)                      */
  uint32_t tstep;          /* static partition tile-size step: 1, else 8      */
  uint32_t body_bpc;       /* body_kernel blocks per CU at most (0: all that fit) */
  uint32_t body_tail;      /* body_kernel unit at the batch's end, packets (0: 16) */
  uint32_t body_engine;    /* body_kernel: 0 by frame size (per-group job
                              sequences for frames under 1 KiB of buffer,
                              else lockstep slots), 1 lockstep, 2 sequences */
  uint32_t walks;          /* 1: every lookup walks the filter table (no key
                              index); 0: the key index answers the keys it
                              holds (DESIGN.md "The key index")              */
} oo_gpu_rx_tuning;
int oo_gpu_rx_set_tuning(oo_gpu_rx_ctx* ctx, const oo_gpu_rx_tuning* t);

/* Device-resident batch: frames, descriptors and results all in HBM.
 * Enqueues the transform of n frames on `stream` and returns immediately.
 * d_counters (device, may be NULL) is incremented per reason.
 * Returns 0 or -EINVAL. */
int oo_gpu_rx_process_dev(oo_gpu_rx_ctx* ctx, const void* d_frames,
                          uint64_t frames_bytes,
                          const oo_gpu_pkt_desc* d_desc, uint32_t n,
                          oo_gpu_rx_result* d_out,
                          oo_gpu_rx_counters* d_counters, void* stream);

/* TX checksum fill on HBM-resident frames, in place, asynchronous on
 * `stream`: for each descriptor, oo_pkt_calc_checksums
 * (src/lib/transport/ip/pkt_checksum.c:20-102) as calc_csum_if_needed
 * (src/lib/transport/ip/netif_tx.c:24-40) runs it on the AF_XDP TX path --
 * TCP and UDP frames only (one 802.1Q tag parsed as on RX): the IPv4 header
 * checksum (ef_ip_checksum, src/lib/ciul/checksum.c:185-212), then the UDP
 * check field (ef_udp_checksum{,_ip6}, :225-250; not for an IPv4 fragment;
 * 0 is sent as 0xffff) or the TCP one (ef_tcp_checksum{,_ip6}, :260-296)
 * over the L4 header and the rest of the frame.  Frames whose headers do not
 * fit, with IHL < 5 or TCP doff < 5 are left as they are where the
 * reference would assert.  The table state of ctx is not used.
 * Returns 0 or -errno. */
int oo_gpu_tx_fill_dev(oo_gpu_rx_ctx* ctx, void* d_frames, uint64_t frames_bytes,
                       const oo_gpu_pkt_desc* d_desc, uint32_t n, void* stream);

/* AF_XDP RX ring entry (struct xdp_desc, <linux/if_xdp.h>). */
typedef struct oo_gpu_xdp_desc {
  uint64_t addr;     /* UMEM offset of the frame's first byte */
  uint32_t len;      /* frame length */
  uint32_t options;  /* not read */
} oo_gpu_xdp_desc;

/* The transform straight off an AF_XDP RX ring, asynchronous on `stream`:
 * n entries from consumer index `cons`, entry i at
 * d_ring[(cons + i) & ring_mask] (ring_mask + 1 a power of two, n at most
 * that), record i to d_out[i].  As efxdp_ef_eventq_poll
 * (src/lib/ciul/efxdp_vi.c:309-358) with netif_event.c:1715-1736 turns an
 * entry into a packet: buffer addr / 2048, frame at offset addr & 2047 --
 * UMEM + addr -- of length len as ef_event's 16-bit rx.len (ef_vi.h:154)
 * carries it, on the ring's interface intf_i.  d_umem / umem_bytes play the
 * frame buffer's part (an entry outside it is an empty frame).  The ring may
 * be device memory or host memory the device can read (hipHostRegister).
 * Returns 0 or -errno. */
int oo_gpu_rx_xdp_dev(oo_gpu_rx_ctx* ctx, const void* d_umem, uint64_t umem_bytes,
                      const oo_gpu_xdp_desc* d_ring, uint32_t ring_mask,
                      uint32_t cons, uint32_t n, int intf_i,
                      oo_gpu_rx_result* d_out, oo_gpu_rx_counters* d_counters,
                      void* stream);

/* One batched poll of an AF_XDP RX ring (efxdp_ef_eventq_poll's RX branch,
 * efxdp_vi.c:316-356, for up to max_n entries instead of evs_len events):
 * reads *consumer and *producer (host words), runs oo_gpu_rx_xdp_dev over
 * the min(producer - consumer, max_n) entries, waits for the stream, then
 * publishes the consumer index (the reference's ci_mb() and store,
 * :352-355) -- only after the device has read the entries.
 * Returns the number of entries consumed or -errno. */
int oo_gpu_rx_xdp_poll(oo_gpu_rx_ctx* ctx, const void* d_umem, uint64_t umem_bytes,
                       const oo_gpu_xdp_desc* d_ring, uint32_t ring_mask,
                       volatile uint32_t* consumer, const volatile uint32_t* producer,
                       uint32_t max_n, int intf_i, oo_gpu_rx_result* d_out,
                       oo_gpu_rx_counters* d_counters, void* stream);

/* Host memory the device may read and write directly (hipHostRegister,
 * mapped): packet-buffer pools / AF_XDP UMEM and rings
 * (efhw/af_xdp.c:463-500 registers the same memory with the kernel),
 * result arrays.  *dev_ptr (may be NULL) receives the device address of p,
 * for oo_gpu_rx_xdp_dev / _poll (zero-copy ingest) or process_dev.
 * Registered frames, descriptors and results skip the pinned staging copy
 * of oo_gpu_rx_submit.
 * The contract, enforced: whole pages -- p and bytes multiples of the page
 * size -- that no other registration of the process (any context) holds;
 * -EINVAL otherwise.  The memory stays mapped until it is unregistered:
 * unregister first, then unmap or free it (a context holding registrations
 * does not close, oo_gpu_rx_close).  Pages of the range should hold nothing
 * the caller copies to or from the device as pageable memory (an mmap'd or
 * huge-page pool, as Onload's is).  A host-only
 * context keeps the same books (*dev_ptr = p).  0, -EINVAL, -ENOMEM,
 * -ENODEV, -EIO.
 * unregister: waits for the context's batches, then 0, -ENOENT (p is not a
 * registered base of this context) or -EIO (the runtime refused: the range
 * stays registered).  registered: the number of ranges the context holds. */
int oo_gpu_rx_host_register(oo_gpu_rx_ctx* ctx, void* p, uint64_t bytes, void** dev_ptr);
int oo_gpu_rx_host_unregister(oo_gpu_rx_ctx* ctx, void* p);
int oo_gpu_rx_host_registered(const oo_gpu_rx_ctx* ctx);

/* Asynchronous host-memory batch (the NIC ring -> socket path): enqueues the
 * H2D copy of frames and descriptors, the transform and the D2H copy of the
 * results (and of the per-reason deltas, if `delta` is not NULL) on one of
 * two staging slots, each with its own stream, so the copies of one batch
 * overlap the transform of the other.  Unregistered buffers go through the
 * slot's pinned staging (a host memcpy at submit for frames/descriptors, at
 * wait for results).  Frame bytes and n must fit the staging sizes given at
 * open.  *ticket identifies the batch.  A submit on a slot still in use
 * completes that slot's batch first (its results land; its wait then
 * returns -ENOENT).  submit: 0 or -errno.  wait: n, -ENOENT (unknown or
 * already completed ticket), -EIO. */
int oo_gpu_rx_submit(oo_gpu_rx_ctx* ctx, const void* frames, uint64_t frames_bytes,
                     const oo_gpu_pkt_desc* desc, uint32_t n, oo_gpu_rx_result* out,
                     oo_gpu_rx_counters* delta, uint64_t* ticket);
int oo_gpu_rx_wait(oo_gpu_rx_ctx* ctx, uint64_t ticket);

/* Asynchronous zero-copy batch: frames, descriptors and results are device
 * addresses -- HBM, or registered host memory (oo_gpu_rx_host_register's
 * dev_ptr: a packet-buffer pool / UMEM read in place, over PCIe) -- and
 * nothing is copied.  Runs on one of the two staging slots' streams like
 * oo_gpu_rx_submit (the context needs host staging; its sizes do not bound
 * this call) and completes with oo_gpu_rx_wait (returns n).  0 or -errno. */
int oo_gpu_rx_submit_mapped(oo_gpu_rx_ctx* ctx, const void* d_frames, uint64_t frames_bytes,
                            const oo_gpu_pkt_desc* d_desc, uint32_t n,
                            oo_gpu_rx_result* d_out, uint64_t* ticket);

/* submit + wait.  Returns n or -errno. */
int oo_gpu_rx_batch(oo_gpu_rx_ctx* ctx, const void* frames,
                    uint64_t frames_bytes, const oo_gpu_pkt_desc* desc,
                    uint32_t n, oo_gpu_rx_result* out,
                    oo_gpu_rx_counters* delta);

/* ---------------------------------------------------------------------
 * Multi-GPU group (SURVEY.md §8(b) "device ids", §8(e)).  Packets are
 * independent and the tables are read-only during a batch, so one stack's
 * batches spread over the GPUs of a node as contiguous shares, one per
 * member; every member holds a replica of the tables, kept identical by
 * applying the same changes in the same order (deterministic placement,
 * return codes included -- oof's single serialisation point,
 * oof_interface.c:184-217); no collective touches the data path.
 *
 * Two shapes.  In one process: oo_gpu_rx_group_open over a device list (a
 * device may repeat, several members on one GPU; a negative device makes a
 * host-only member), the calling thread driving every member.  Across
 * processes, one per GPU: rank 0 makes an id (oo_gpu_rx_group_rccl_id), the
 * caller's control plane hands its OO_GPU_RX_GROUP_ID_BYTES to every rank,
 * each joins with its rank (one local member on cfg->device) and RCCL over
 * xGMI carries the table image, the changes and the records (librccl is
 * loaded at the first join: -ENOSYS without it).
 * --------------------------------------------------------------------- */
#define OO_GPU_RX_GROUP_ID_BYTES 128

typedef struct oo_gpu_rx_group oo_gpu_rx_group;

/* One member's share of a batch: its frames, descriptors, records and
 * (optional) counters in its device's memory, and its stream. */
typedef struct oo_gpu_rx_shard {
  const void*             d_frames;
  uint64_t                frames_bytes;
  const oo_gpu_pkt_desc*  d_desc;
  uint32_t                n;
  uint32_t                rsvd;
  oo_gpu_rx_result*       d_out;
  oo_gpu_rx_counters*     d_counters;   /* may be NULL */
  void*                   stream;
} oo_gpu_rx_shard;

/* n members (<= 64), member i a context opened with cfg on devices[i]. */
int  oo_gpu_rx_group_open(oo_gpu_rx_group** out, const oo_gpu_rx_cfg* cfg,
                          const int32_t* devices, uint32_t n);
int  oo_gpu_rx_group_rccl_id(void* id);
int  oo_gpu_rx_group_join(oo_gpu_rx_group** out, const oo_gpu_rx_cfg* cfg, uint32_t rank,
                          uint32_t nranks, const void* id);
/* The join shape over a caller's transport instead of RCCL: a host-only
 * member (cfg->device < 0, else -EINVAL) whose collectives move host memory
 * through the four calls below -- the control plane's own channel between
 * the processes of a stack, for replicating its tables without a GPU, and
 * the harness that runs the collectives' sequencing with injected failures.
 * Each call is collective over the nranks callers and returns 0 or -errno
 * locally: bcast copies rank 0's `bytes` at p to every rank's p; max_u32 /
 * sum_u32 reduce n words in place; gather moves every rank's `bytes` at src
 * to rank 0's dst in rank order (bytes_of[k]: rank k's bytes, the same on
 * every rank). */
typedef struct oo_gpu_rx_group_transport {
  void* arg;
  int (*bcast)(void* arg, void* p, uint64_t bytes);
  int (*max_u32)(void* arg, uint32_t* v, uint32_t n);
  int (*sum_u32)(void* arg, uint32_t* v, uint32_t n);
  int (*gather)(void* arg, const void* src, uint64_t bytes, void* dst, const uint64_t* bytes_of);
} oo_gpu_rx_group_transport;
int  oo_gpu_rx_group_join_transport(oo_gpu_rx_group** out, const oo_gpu_rx_cfg* cfg, uint32_t rank,
                                    uint32_t nranks, const oo_gpu_rx_group_transport* t);
/* 0, or -EBUSY (nothing closed) while a member holds registered host memory. */
int  oo_gpu_rx_group_close(oo_gpu_rx_group* g);
/* Local members, this process's rank (0 in one process), member i's context
 * (its own calls -- export, sync_tables, stream_done -- work as for any
 * context; table changes go through the group). */
uint32_t       oo_gpu_rx_group_size(const oo_gpu_rx_group* g);
uint32_t       oo_gpu_rx_group_rank(const oo_gpu_rx_group* g);
oo_gpu_rx_ctx* oo_gpu_rx_group_member(oo_gpu_rx_group* g, uint32_t i);
/* Table changes on every local member in call order; the members' common
 * return code (-EIO if a replica disagrees).  Across processes only rank 0
 * changes the tables (-EPERM elsewhere); the changes reach the other ranks
 * with oo_gpu_rx_group_share_ops. */
int oo_gpu_rx_group_table_insert(oo_gpu_rx_group* g, int af, const void* laddr,
                                 uint16_t lport_be16, const void* raddr, uint16_t rport_be16,
                                 uint8_t protocol, int32_t sock_id);
int oo_gpu_rx_group_table_remove(oo_gpu_rx_group* g, int af, const void* laddr,
                                 uint16_t lport_be16, const void* raddr, uint16_t rport_be16,
                                 uint8_t protocol, int32_t sock_id);
int oo_gpu_rx_group_sock_set(oo_gpu_rx_group* g, int32_t sock_id, const oo_gpu_rx_sock* sock);
/* Byte-balanced contiguous split of n packets (host descriptors) into
 * `parts` shares: first[0..parts], share k = [first[k], first[k+1]), each
 * holding about the same algorithmic bytes (frame + 16-B descriptor + 32-B
 * record). */
int oo_gpu_rx_group_split(const oo_gpu_rx_group* g, const oo_gpu_pkt_desc* desc, uint32_t n,
                          uint32_t parts, uint32_t* first);
/* In one process: member i transforms shards[i], asynchronously on its
 * stream (oo_gpu_rx_process_dev): work the caller queued on other streams
 * (the fill of a shard's buffers) must be ordered before it by the caller. */
int oo_gpu_rx_group_process(oo_gpu_rx_group* g, const oo_gpu_rx_shard* shards);
/* In one process, after process: the members' records into dst (sum of
 * the shards' n, member order; device or host memory, NULL: none), each
 * copied on its member's stream; then waits for every member and sums the
 * counters into *counters (host, may be NULL). */
int oo_gpu_rx_group_gather(oo_gpu_rx_group* g, const oo_gpu_rx_shard* shards,
                           oo_gpu_rx_result* dst, oo_gpu_rx_counters* counters);
/* Across processes (every rank calls each, collectively): rank 0's tables
 * to every rank (one image broadcast); rank 0's changes since then, applied
 * by the others in order (returns how many; -EIO on every rank when a
 * replica's return code differs from rank 0's or rank 0 lost a change, and
 * the caller then shares the tables again); every rank's n records to
 * rank 0's d_dst in rank order (rank 0 passes counts[nranks]; a count
 * that differs from its rank's n, or rank 0 without d_dst / counts, is
 * -EINVAL on every rank and moves nothing); the device counters summed on
 * every rank.  Each call enters all of its collectives on every rank: where
 * a local failure would leave a rank out of the next one, every rank first
 * agrees on it (a one-word maximum) and all return the error together;
 * later local failures are reported after the last collective.  The
 * staging they use is allocated at the join.  A joined group of one rank
 * runs the same RCCL calls.  A failure of the agreement itself (-EIO)
 * means the communicator is unusable: close the group. */
int oo_gpu_rx_group_share_tables(oo_gpu_rx_group* g, void* stream);
int oo_gpu_rx_group_share_ops(oo_gpu_rx_group* g, void* stream);
int oo_gpu_rx_group_gather_rccl(oo_gpu_rx_group* g, const oo_gpu_rx_result* d_out, uint32_t n,
                                oo_gpu_rx_result* d_dst, const uint32_t* counts, void* stream);
int oo_gpu_rx_group_sum_counters(oo_gpu_rx_group* g, oo_gpu_rx_counters* d_counters,
                                 void* stream);
/* 1 when the group's collectives run over RCCL (a joined group, any number
 * of ranks), 0 for a group opened in one process. */
int oo_gpu_rx_group_uses_rccl(const oo_gpu_rx_group* g);

/* ---------------------------------------------------------------------
 * Host-pure checksum verifiers: the reference's public C API for this path
 * (src/include/etherfabric/checksum.h:246-308, src/lib/ciul/checksum.c:
 * 298-351) and ci_ip_csum_correct (netif_event.c:80-94), same argument
 * shapes and verdicts (non-zero = correct).  No GPU, no state, no
 * allocation: thread-safe.  Headers are the wire headers (glibc
 * struct iphdr / udphdr / tcphdr, linux struct ipv6hdr); iov describes the
 * L4 payload after the UDP header / the TCP header of doff*4 bytes, its
 * elements paired across boundaries as ip_csum64_partialv (:134-159).
 * As in the reference, an IPv4 UDP check field of 0 means "no checksum" to
 * the caller (udp_rx.c:111-117), not to these functions. */
struct iphdr;
struct ipv6hdr;
struct udphdr;
struct tcphdr;
struct iovec;
int oo_rx_ip_csum_ok(const struct iphdr* ip, int max_ip_len);
int oo_rx_udp_csum_ok(const struct iphdr* ip, const struct udphdr* udp,
                      const struct iovec* iov, int iovlen);
int oo_rx_udp_csum_ok_ip6(const struct ipv6hdr* ip6, const struct udphdr* udp,
                          const struct iovec* iov, int iovlen);
int oo_rx_tcp_csum_ok(const struct iphdr* ip, const struct tcphdr* tcp,
                      const struct iovec* iov, int iovlen);
int oo_rx_tcp_csum_ok_ip6(const struct ipv6hdr* ip6, const struct tcphdr* tcp,
                          const struct iovec* iov, int iovlen);
int oo_rx_udp_csum_ok_ipx(int af, const void* ipx, const struct udphdr* udp,
                          const void* payload, size_t payload_len);
int oo_rx_tcp_csum_ok_ipx(int af, const void* ipx, const struct tcphdr* tcp,
                          const void* payload, size_t payload_len);

/* Reason code -> short name ("DELIVER", "UDP_CSUM", ...). */
const char* oo_gpu_rx_reason_str(int reason);

#ifdef __cplusplus
}
#endif

#endif /* OO_GPU_RX_H */
