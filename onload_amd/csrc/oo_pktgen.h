/* SPDX-License-Identifier: BSD-2-Clause */
/*
 * oo_pktgen.h -- seeded synthetic frame generator for the BASELINE.json
 * configurations.  Frame construction follows the pattern
 * of the reference's ef_vi sample senders (src/tests/ef_vi/utils.c); the
 * checksums are filled the way the AF_XDP TX path does
 * (src/lib/transport/ip/pkt_checksum.c:20-102).
 *
 * Packet i of a configuration depends only on (config, seed, i), so any
 * packet range can be generated independently (one shard per GPU rank).
 */
#ifndef OO_PKTGEN_H
#define OO_PKTGEN_H

#include <stdint.h>
#include "../../include/oo_gpu_rx.h"

#ifdef __cplusplus
extern "C" {
#endif

enum {
  OO_PG_CFG_UDP1514 = 2,   /* 1514-byte IPv4/UDP                              */
  OO_PG_CFG_UDP64 = 3,     /* 64-byte IPv4/UDP                                */
  OO_PG_CFG_TCPMIX = 4,    /* IPv4/TCP 64..9014 B log-uniform, IP+TCP options */
  OO_PG_CFG_IMIX = 5       /* IMIX 64:594:1518, TCP+UDP, IPv4+IPv6            */
};

/* One filter-table insert the configuration's world needs. */
typedef struct oo_pg_filter {
  int32_t sock;
  uint8_t af;        /* 4 or 6 */
  uint8_t proto;
  uint16_t lport_be;
  uint16_t rport_be;
  uint8_t raddr_any; /* raddr is the wildcard */
  uint8_t rsvd;
  uint8_t laddr[16]; /* 4 or 16 bytes used */
  uint8_t raddr[16];
} oo_pg_filter;

/* Default seed of a configuration: 0x4F4E4C44000000NN. */
uint64_t oo_pg_default_seed(int config);

/* The socket world: fills up to max_filters filters and the socket records
 * (socks[0..*n_socks-1]).  Returns the number of filters, or -1. */
int oo_pg_world(int config, oo_pg_filter* filters, int max_filters,
                oo_gpu_rx_sock* socks, int max_socks, int* n_socks);

/* Frame length of packet i. */
uint32_t oo_pg_len(int config, uint64_t seed, uint64_t i);

/* Bytes needed to pack packets [first, first+n) at `align`-byte alignment. */
uint64_t oo_pg_bytes(int config, uint64_t seed, uint64_t first, uint32_t n,
                     uint32_t align);

/* Generate packets [first, first+n) packed at `align`-byte aligned offsets
 * from buf[0]; writes n descriptors (frame_off relative to buf).  Returns the
 * bytes used, or 0 if cap is too small.  nthreads > 1 generates in
 * parallel. */
uint64_t oo_pg_gen(int config, uint64_t seed, uint64_t first, uint32_t n,
                   uint32_t align, uint8_t* buf, uint64_t cap,
                   oo_gpu_pkt_desc* desc, int nthreads);

/* Byte-balanced shard boundaries of packets [0, n_total) over `world`
 * ranks: firsts[0..world] (rank r owns [firsts[r], firsts[r+1])).  0 or -1. */
int oo_pg_split(int config, uint64_t seed, uint64_t n_total, int world, uint32_t align,
                uint64_t* firsts, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
