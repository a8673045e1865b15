/* SPDX-License-Identifier: BSD-2-Clause */
/*
 * rx_oracle.h -- CPU restatement of Onload's software RX transform.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (onload_amd/, include/)
 * may include, link or call this.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg use it, and only as the checker / the CPU
 * baseline.  See oracle/rx_oracle.c for the per-function reference citations
 * and DESIGN.md "Oracle and parity pinning" for how it is pinned.
 */
#ifndef OO_RX_ORACLE_H
#define OO_RX_ORACLE_H

#include <stddef.h>
#include <stdint.h>
#include "../include/oo_gpu_rx.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oo_or_tables oo_or_tables;

oo_or_tables* oo_or_tables_new(int ip4_log2, int ip6_log2, uint32_t max_socks,
                               const uint8_t* intf_hwport, int n_intf);
void oo_or_tables_free(oo_or_tables* t);
oo_or_tables* oo_or_tables_clone(const oo_or_tables* t);
int  oo_or_insert(oo_or_tables* t, int af, const void* laddr, uint16_t lport,
                  const void* raddr, uint16_t rport, uint8_t proto, int32_t id);
int  oo_or_remove(oo_or_tables* t, int af, const void* laddr, uint16_t lport,
                  const void* raddr, uint16_t rport, uint8_t proto, int32_t id);
int  oo_or_lookup(const oo_or_tables* t, int af, const void* laddr,
                  uint16_t lport, const void* raddr, uint16_t rport,
                  uint8_t proto);
int  oo_or_slot(const oo_or_tables* t, int af, uint32_t slot,
                uint32_t* id_state, int32_t* route_count, uint16_t* lport);
int  oo_or_sock_set(oo_or_tables* t, int32_t id, const oo_gpu_rx_sock* s);
uint32_t oo_or_dump(const oo_or_tables* t, int64_t* rows, uint32_t cap);

/* One IPv4 lookup stage (ci_netif_filter_for_each_match): matches, first. */
int  oo_or_walk4(const oo_or_tables* t, uint32_t la, uint32_t lp, uint32_t ra, uint32_t rp,
                 uint32_t proto, int intf_i, int vlan, int stop, int32_t* first);
/* One frame: the whole handle_rx_csum_bad -> handle_rx_pkt -> L4 demux. */
void oo_or_rx_one(const oo_or_tables* t, const uint8_t* frame, int len,
                  int intf_i, oo_gpu_rx_result* out);
/* A batch over `nthreads` host threads (contiguous shards); a descriptor
 * outside [0, frames_bytes) is an empty frame. */
void oo_or_rx_batch(const oo_or_tables* t, const uint8_t* frames,
                    uint64_t frames_bytes, const oo_gpu_pkt_desc* desc, uint32_t n,
                    oo_gpu_rx_result* out, int nthreads);

/* The batch straight off an AF_XDP RX ring (efxdp_vi.c:316-356). */
void oo_or_xdp_batch(const oo_or_tables* t, const uint8_t* umem,
                     uint64_t umem_bytes, const oo_gpu_xdp_desc* ring,
                     uint32_t mask, uint32_t cons, uint32_t n, int intf_i,
                     oo_gpu_rx_result* out);

/* Checksum verifiers with the reference's argument shapes
 * (checksum.c:298-351, netif_event.c:80-94) for pinning against the
 * compiled reference. */
int oo_or_ip4_hdr_ok(const uint8_t* ip, int max_ip_len);
int oo_or_udp4_ok(const uint8_t* ip4, const uint8_t* udp,
                  const uint8_t* pay, size_t paylen);
int oo_or_udp6_ok(const uint8_t* ip6, const uint8_t* udp,
                  const uint8_t* pay, size_t paylen);
int oo_or_tcp4_ok(const uint8_t* ip4, const uint8_t* tcp,
                  const uint8_t* pay, size_t paylen);
int oo_or_tcp6_ok(const uint8_t* ip6, const uint8_t* tcp,
                  const uint8_t* pay, size_t paylen);

/* TX checksum fill (pkt_checksum.c:20-102), in place. */
void oo_or_tx_fill_one(uint8_t* frame, int len);
void oo_or_tx_fill_batch(uint8_t* frames, uint64_t frames_bytes,
                         const oo_gpu_pkt_desc* desc, uint32_t n);

/* Hashes (src/include/onload/hash.h). */
uint32_t oo_or_hash3(uint32_t laddr, uint32_t lport, uint32_t raddr,
                     uint32_t rport, uint32_t proto);
uint32_t oo_or_hash1(uint32_t mask, uint32_t laddr, uint32_t lport,
                     uint32_t raddr, uint32_t rport, uint32_t proto);
uint32_t oo_or_hash2(uint32_t laddr, uint32_t lport, uint32_t raddr,
                     uint32_t rport, uint32_t proto);
uint32_t oo_or_addr_xor(const uint8_t* a16);

#ifdef __cplusplus
}
#endif
#endif
