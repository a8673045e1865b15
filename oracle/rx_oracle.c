/* SPDX-License-Identifier: BSD-2-Clause */
/*
 * rx_oracle.c -- CPU restatement of Onload's software RX transform
 * (checksum verify + header parse + 4-tuple socket demux).
 *
 * TEST INFRASTRUCTURE ONLY: this is the checker the GPU library is compared
 * against and the CPU baseline bench.py times.  The product never links it.
 *
 * It restates, in the reference's check order, the behaviour of
 *   handle_rx_csum_bad        src/lib/transport/ip/netif_event.c:1014-1128
 *   ci_parse_rx_vlan          netif_event.c:116-132
 *   ci_ip_csum_correct        netif_event.c:80-94
 *   ci_tcp_csum_correct       netif_event.c:97-113
 *   ci_udp_csum_correct       src/lib/transport/ip/udp_rx.c:101-121
 *   handle_rx_pkt             netif_event.c:250-451
 *   ci_ip_options_parse       netif_event.c:135-185
 *   ci_udp_handle_rx          udp_rx.c:236-307 (+ deliver rule :141-228)
 *   ci_tcp_handle_rx          src/lib/transport/ip/tcp_rx.c:4681-4836
 *   filter table lookup/insert/remove
 *                             src/lib/transport/ip/netif_table.c:86-503,
 *                             netif_table_ip6.c:13-345, hash.h:31-173
 *   checksum arithmetic       src/lib/ciul/checksum.c:53-351,
 *                             src/lib/citools/ip_csum_partial.c:20-39,
 *                             src/include/ci/tools/ipcsum_base.h:10-14
 *
 * Pinning (DESIGN.md "Oracle and parity pinning"): the checksum verifiers and
 * the hashes are checked bit-for-bit against the reference's own compiled
 * checksum.c / ip_csum_partial.c / hash.h (oracle/_ref, built by
 * oracle/Makefile) and the reference unit test's known answers
 * (src/tests/unit/lib/ciul/checksum.c:13-62); the gate order, lookup order and
 * outcomes against the reference runs recorded in SURVEY.md §8(c) and the
 * lookup-order unit test (src/tests/unit/lib/transport/ip/tcp_rx.c:30-70).
 *
 * Byte reads beyond the frame length return 0 (the reference reads whatever
 * follows in the packet buffer; only frames shorter than 16 bytes, which are
 * always dropped SHORT_L2, can differ, and only in the recorded vlan field).
 */
#include "rx_oracle.h"

#include <errno.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ */
/* Byte access helpers.                                                */

typedef struct { const uint8_t* p; int len; } frame_t;

static inline unsigned rd8(frame_t f, int i)
{ return (i >= 0 && i < f.len) ? f.p[i] : 0u; }
/* Network-order 16-bit value held in a host integer (LE load). */
static inline unsigned rd16n(frame_t f, int i)
{ return rd8(f, i) | (rd8(f, i + 1) << 8); }
/* Host-order value of a BE16 field (CI_BSWAP_BE16 of the above). */
static inline unsigned be16(frame_t f, int i)
{ return (rd8(f, i) << 8) | rd8(f, i + 1); }
static inline uint32_t rd32n(frame_t f, int i)
{ return rd16n(f, i) | ((uint32_t)rd16n(f, i + 2) << 16); }

static inline uint32_t bswap32(uint32_t x)
{ return __builtin_bswap32(x); }

/* ------------------------------------------------------------------ */
/* RFC 1071 arithmetic.
 *
 * The reference accumulates little-endian 64/32/16-bit loads with
 * end-around carry (checksum.c:87-174) or plain 32-bit sums of LE u16 words
 * (ip_csum_partial.c:20-39) and folds to 16 bits.  Every one of those steps
 * preserves the value mod 0xffff and never turns a non-zero value into 0, so
 * "the folded complement is 0" <=> "the exact integer sum S of the LE u16
 * words (an odd last byte as a low byte) is non-zero and S = 0 mod 0xffff".
 * Here S is kept exactly in 64 bits (no carry needed below 2^48 bytes). */

/* Exact sum of LE u16 words over n bytes at p; an odd final byte is the low
 * byte of a word padded with zero (ip_csum_partial.c:33-36,
 * checksum.c:150-156). */
static uint64_t sum16(const uint8_t* p, size_t n)
{
  /* 8 bytes per step (as ip_csum64_partial, checksum.c:87-131, loads 8 B):
   * the four words go to two 32-bit lanes of two accumulators, each lane
   * gaining < 2^16 per step, so no lane overflows below 2^16 steps
   * (512 KiB; a frame is < 64 KiB). */
  uint64_t a = 0, b = 0, s;
  size_t i = 0;
  for( ; i + 8 <= n; i += 8 ) {
    uint64_t w;
    memcpy(&w, p + i, 8);
    a += w & 0x0000ffff0000ffffull;
    b += (w >> 16) & 0x0000ffff0000ffffull;
  }
  s = (a & 0xffffffffu) + (a >> 32) + (b & 0xffffffffu) + (b >> 32);
  for( ; i + 4 <= n; i += 4 ) {
    uint32_t w;
    memcpy(&w, p + i, 4);
    s += (w & 0xffffu) + (w >> 16);
  }
  for( ; i + 2 <= n; i += 2 )
    s += (uint32_t)p[i] | ((uint32_t)p[i + 1] << 8);
  if( i < n )
    s += p[i];
  return s;
}

/* Fold to 16 bits with end-around carry. */
static inline uint32_t fold16(uint64_t s)
{
  while( s >> 16 )
    s = (s & 0xffffu) + (s >> 16);
  return (uint32_t)s;
}

/* ~fold == 0, i.e. the verifier's "csum == 0" test. */
static inline int folded_ok(uint64_t s)
{ return s != 0 && fold16(s) == 0xffffu; }

/* ci_ip_csum_correct (netif_event.c:80-94): IHL/tot_len bounds, then
 * ci_ip_csum_partial over 4*IHL bytes + ci_ip_hdr_csum_finish. */
int oo_or_ip4_hdr_ok(const uint8_t* ip, int max_ip_len)
{
  int ihl4 = (ip[0] & 0xf) * 4;
  int ip_len = (ip[2] << 8) | ip[3];
  if( max_ip_len < ihl4 || max_ip_len < ip_len )
    return 0;
  return folded_ok(sum16(ip, (size_t)ihl4));
}

/* IPv4 pseudo-header words: saddr + daddr as LE u32 (checksum.c:304-305),
 * i.e. four LE u16 words. */
static inline uint64_t ip4_addr_sum(const uint8_t* ip4)
{ return sum16(ip4 + 12, 8); }

/* ef_udp_checksum_is_correct (checksum.c:298-311): pseudo-header
 * saddr+daddr+htons(17)+udp->len, the 8-byte header (check included), the
 * payload iovec. */
int oo_or_udp4_ok(const uint8_t* ip4, const uint8_t* udp,
                  const uint8_t* pay, size_t paylen)
{
  uint64_t s = ip4_addr_sum(ip4) + 0x1100u + (udp[4] | (udp[5] << 8));
  s += sum16(udp, 8) + sum16(pay, paylen);
  return folded_ok(s);
}

/* ef_ip6_pseudo_hdr_checksum (checksum.c:215-223): 32 address bytes +
 * len_be16 + htonl(proto). */
static inline uint64_t ip6_pseudo(const uint8_t* ip6, unsigned len_n,
                                  unsigned proto)
{ return sum16(ip6 + 8, 32) + len_n + ((uint64_t)proto << 8); }

/* ef_udp_checksum_ip6_is_correct (checksum.c:313-324). */
int oo_or_udp6_ok(const uint8_t* ip6, const uint8_t* udp,
                  const uint8_t* pay, size_t paylen)
{
  uint64_t s = ip6_pseudo(ip6, udp[4] | (udp[5] << 8), 17);
  s += sum16(udp, 8) + sum16(pay, paylen);
  return folded_ok(s);
}

/* ef_tcp_checksum_is_correct (checksum.c:326-339): pseudo-header length is
 * (u16)(tot_len - 4*IHL) from the IP header; the header covers doff*4 bytes. */
int oo_or_tcp4_ok(const uint8_t* ip4, const uint8_t* tcp,
                  const uint8_t* pay, size_t paylen)
{
  unsigned tot = (ip4[2] << 8) | ip4[3];
  unsigned ihl4 = (ip4[0] & 0xf) * 4u;
  unsigned plen = (tot - ihl4) & 0xffffu;
  /* htonl(6<<16 | plen) as an LE u32 = two LE u16 words: 0x0600 and the
   * byte-swapped plen. */
  uint64_t s = ip4_addr_sum(ip4) + 0x0600u + (((plen & 0xff) << 8) | (plen >> 8));
  s += sum16(tcp, ((tcp[12] & 0xf0u) >> 2)) + sum16(pay, paylen);
  return folded_ok(s);
}

/* ef_tcp_checksum_ip6_is_correct (checksum.c:341-351). */
int oo_or_tcp6_ok(const uint8_t* ip6, const uint8_t* tcp,
                  const uint8_t* pay, size_t paylen)
{
  uint64_t s = ip6_pseudo(ip6, ip6[4] | (ip6[5] << 8), 6);
  s += sum16(tcp, ((tcp[12] & 0xf0u) >> 2)) + sum16(pay, paylen);
  return folded_ok(s);
}

/* ------------------------------------------------------------------ */
/* Hashes: src/include/onload/hash.h:31-42, 84-93, 137-144, 165-173.
 * All inputs are network-order values held in host integers; on a
 * little-endian host CI_BSWAP_LE32 is the identity and CI_BSWAP_BE32 a
 * byte swap. */

uint32_t oo_or_hash3(uint32_t laddr, uint32_t lport, uint32_t raddr,
                     uint32_t rport, uint32_t proto)
{
  uint32_t h = bswap32(raddr) ^ laddr ^ ((rport << 16) | lport) ^ proto;
  h ^= h >> 16;
  h ^= h >> 8;
  return h;
}

uint32_t oo_or_hash1(uint32_t mask, uint32_t laddr, uint32_t lport,
                     uint32_t raddr, uint32_t rport, uint32_t proto)
{ return oo_or_hash3(laddr, lport, raddr, rport, proto) & mask; }

uint32_t oo_or_hash2(uint32_t laddr, uint32_t lport, uint32_t raddr,
                     uint32_t rport, uint32_t proto)
{ return ((laddr ^ raddr) ^ ((lport << 16) | rport) ^ proto) | 1u; }

uint32_t oo_or_addr_xor(const uint8_t* a)
{
  uint32_t x = 0, w;
  int i;
  if( a == NULL )
    return 0;
  for( i = 0; i < 4; ++i ) {
    memcpy(&w, a + 4 * i, 4);
    x ^= w;
  }
  return x;
}

/* ------------------------------------------------------------------ */
/* Filter-table mirror.                                                 */

/* IPv4 entry state in the top two bits of id_state (netif_table.c:34-42). */
#define ST_MASK      0xc0000000u
#define ID_MASK      0x3fffffffu
#define ST_PREFERRED 0x00000000u
#define ST_REHASHED  0x40000000u
#define ST_EMPTY     0x80000000u
#define ST_TOMBSTONE 0xc0000000u
#define OCCUPIED(s)  (((~(s)) & ST_EMPTY & ST_TOMBSTONE) != 0)

/* IPv6 id sentinels (netif_table_ip6.c:10-11). */
#define ID6_TOMBSTONE (-1)
#define ID6_EMPTY     (-2)

typedef struct { int32_t id; int32_t route_count; uint8_t laddr[16]; } ip6e_t;

struct oo_or_tables {
  uint32_t  ip4_mask;
  uint32_t* ip4_id_state;
  uint32_t* ip4_laddr;
  int32_t*  ip4_route;
  uint16_t* ip4_lport;
  uint32_t  ip6_mask;
  ip6e_t*   ip6;
  uint32_t  max_socks;
  oo_gpu_rx_sock* socks;
  uint8_t   hwport[OO_GPU_RX_MAX_INTF];
};

oo_or_tables* oo_or_tables_new(int ip4_log2, int ip6_log2, uint32_t max_socks,
                               const uint8_t* intf_hwport, int n_intf)
{
  oo_or_tables* t;
  uint32_t n4, n6, i;
  if( ip4_log2 < 16 || ip4_log2 > 24 || ip6_log2 < 1 || ip6_log2 > 24 ||
      max_socks == 0 || n_intf < 0 || n_intf > OO_GPU_RX_MAX_INTF )
    return NULL;
  t = calloc(1, sizeof(*t));
  n4 = 1u << ip4_log2;
  n6 = 1u << ip6_log2;
  t->ip4_mask = n4 - 1;
  t->ip6_mask = n6 - 1;
  t->max_socks = max_socks;
  t->ip4_id_state = calloc(n4, 4);
  t->ip4_laddr = calloc(n4, 4);
  t->ip4_route = calloc(n4, 4);
  t->ip4_lport = calloc(n4, 2);
  t->ip6 = calloc(n6, sizeof(ip6e_t));
  t->socks = calloc(max_socks, sizeof(oo_gpu_rx_sock));
  /* ci_netif_filter_init (netif_table.c:592-611), ci_ip6_netif_filter_init
   * (netif_table_ip6.c:349-365). */
  for( i = 0; i < n4; ++i )
    t->ip4_id_state[i] = ST_EMPTY;
  for( i = 0; i < n6; ++i )
    t->ip6[i].id = ID6_EMPTY;
  memset(t->hwport, 0xff, sizeof(t->hwport));
  if( intf_hwport != NULL )
    memcpy(t->hwport, intf_hwport, (size_t)n_intf);
  return t;
}

void oo_or_tables_free(oo_or_tables* t)
{
  if( t == NULL )
    return;
  free(t->ip4_id_state); free(t->ip4_laddr); free(t->ip4_route);
  free(t->ip4_lport); free(t->ip6); free(t->socks); free(t);
}

oo_or_tables* oo_or_tables_clone(const oo_or_tables* t)
{
  oo_or_tables* c = calloc(1, sizeof(*c));
  uint32_t n4 = t->ip4_mask + 1, n6 = t->ip6_mask + 1;
  *c = *t;
  c->ip4_id_state = malloc(n4 * 4u); memcpy(c->ip4_id_state, t->ip4_id_state, n4 * 4u);
  c->ip4_laddr = malloc(n4 * 4u);    memcpy(c->ip4_laddr, t->ip4_laddr, n4 * 4u);
  c->ip4_route = malloc(n4 * 4u);    memcpy(c->ip4_route, t->ip4_route, n4 * 4u);
  c->ip4_lport = malloc(n4 * 2u);    memcpy(c->ip4_lport, t->ip4_lport, n4 * 2u);
  c->ip6 = malloc(n6 * sizeof(ip6e_t)); memcpy(c->ip6, t->ip6, n6 * sizeof(ip6e_t));
  c->socks = malloc(t->max_socks * sizeof(oo_gpu_rx_sock));
  memcpy(c->socks, t->socks, t->max_socks * sizeof(oo_gpu_rx_sock));
  return c;
}

int oo_or_sock_set(oo_or_tables* t, int32_t id, const oo_gpu_rx_sock* s)
{
  if( id < 0 || (uint32_t)id >= t->max_socks || s == NULL )
    return -EINVAL;
  t->socks[id] = *s;
  return 0;
}

static inline uint32_t ld32(const void* p)
{ uint32_t v; memcpy(&v, p, 4); return v; }

/* ci_ip4_netif_filter_insert (netif_table.c:323-406). */
static int ip4_insert(oo_or_tables* t, int32_t id, uint32_t la, uint32_t lp,
                      uint32_t ra, uint32_t rp, uint32_t proto)
{
  uint32_t h1 = oo_or_hash1(t->ip4_mask, la, lp, ra, rp, proto);
  uint32_t h2 = oo_or_hash2(la, lp, ra, rp, proto);
  uint32_t first = h1;
  while( OCCUPIED(t->ip4_id_state[h1]) ) {
    ++t->ip4_route[h1];
    h1 = (h1 + h2) & t->ip4_mask;
    if( h1 == first )
      return -ENOBUFS;   /* the route counts stay incremented, as in :349-376 */
  }
  t->ip4_id_state[h1] = (h1 == first ? ST_PREFERRED : ST_REHASHED) |
                        ((uint32_t)id & ID_MASK);
  t->ip4_laddr[h1] = la;
  t->ip4_lport[h1] = (uint16_t)lp;
  return 0;
}

/* ci_ip4_netif_filter_remove + __ci_ip4_netif_filter_remove
 * (netif_table.c:409-495). */
static void ip4_remove(oo_or_tables* t, int32_t id, uint32_t la, uint32_t lp,
                       uint32_t ra, uint32_t rp, uint32_t proto)
{
  uint32_t h1 = oo_or_hash1(t->ip4_mask, la, lp, ra, rp, proto);
  uint32_t h2 = oo_or_hash2(la, lp, ra, rp, proto);
  uint32_t first = h1, i = h1;
  int hops = 0, k;
  while( 1 ) {
    uint32_t st = t->ip4_id_state[i];
    if( OCCUPIED(st) && (st & ID_MASK) == ((uint32_t)id & ID_MASK) ) {
      if( la == t->ip4_laddr[i] )
        break;
    }
    else if( (st & ST_MASK) == ST_EMPTY )
      return;
    i = (i + h2) & t->ip4_mask;
    ++hops;
    if( i == first )
      return;
  }
  i = h1;
  for( k = 0; k < hops; ++k ) {
    if( --t->ip4_route[i] == 0 && (t->ip4_id_state[i] & ST_MASK) == ST_TOMBSTONE )
      t->ip4_id_state[i] = (t->ip4_id_state[i] & ID_MASK) | ST_EMPTY;
    i = (i + h2) & t->ip4_mask;
  }
  t->ip4_id_state[i] = (t->ip4_id_state[i] & ID_MASK) |
                       (t->ip4_route[i] == 0 ? ST_EMPTY : ST_TOMBSTONE);
}

/* ci_ip6_netif_filter_insert (netif_table_ip6.c:192-262). */
static int ip6_insert(oo_or_tables* t, int32_t id, const uint8_t* la,
                      uint32_t lp, const uint8_t* ra, uint32_t rp,
                      uint32_t proto)
{
  uint32_t lx = oo_or_addr_xor(la), rx = oo_or_addr_xor(ra);
  uint32_t h1 = oo_or_hash1(t->ip6_mask, lx, lp, rx, rp, proto);
  uint32_t h2 = oo_or_hash2(lx, lp, rx, rp, proto);
  uint32_t first = h1;
  while( t->ip6[h1].id >= 0 ) {
    ++t->ip6[h1].route_count;
    h1 = (h1 + h2) & t->ip6_mask;
    if( h1 == first )
      return -ENOBUFS;
  }
  t->ip6[h1].id = id;
  memcpy(t->ip6[h1].laddr, la, 16);
  return 0;
}

/* ci_ip6_netif_filter_remove + __ci_ip6_netif_filter_remove
 * (netif_table_ip6.c:264-345). */
static void ip6_remove(oo_or_tables* t, int32_t id, const uint8_t* la,
                       uint32_t lp, const uint8_t* ra, uint32_t rp,
                       uint32_t proto)
{
  uint32_t lx = oo_or_addr_xor(la), rx = oo_or_addr_xor(ra);
  uint32_t h1 = oo_or_hash1(t->ip6_mask, lx, lp, rx, rp, proto);
  uint32_t h2 = oo_or_hash2(lx, lp, rx, rp, proto);
  uint32_t first = h1, i = h1;
  int hops = 0, k;
  while( 1 ) {
    ip6e_t* e = &t->ip6[i];
    if( e->id == id ) {
      if( memcmp(la, e->laddr, 16) == 0 )
        break;
    }
    else if( e->id == ID6_EMPTY )
      return;
    i = (i + h2) & t->ip6_mask;
    ++hops;
    if( i == first )
      return;
  }
  i = h1;
  for( k = 0; k < hops; ++k ) {
    ip6e_t* e = &t->ip6[i];
    if( --e->route_count == 0 && e->id == ID6_TOMBSTONE )
      e->id = ID6_EMPTY;
    i = (i + h2) & t->ip6_mask;
  }
  t->ip6[i].id = t->ip6[i].route_count == 0 ? ID6_EMPTY : ID6_TOMBSTONE;
}

static const uint8_t zero16[16];

int oo_or_insert(oo_or_tables* t, int af, const void* laddr, uint16_t lport,
                 const void* raddr, uint16_t rport, uint8_t proto, int32_t id)
{
  if( laddr == NULL || id < 0 || (uint32_t)id >= t->max_socks )
    return -EINVAL;
  if( af == 4 )
    return ip4_insert(t, id, ld32(laddr), lport, raddr ? ld32(raddr) : 0,
                      rport, proto);
  if( af == 6 )
    /* ci_netif_filter_insert maps an any raddr to addr_any (:451-453). */
    return ip6_insert(t, id, laddr, lport, raddr ? raddr : zero16, rport,
                      proto);
  return -EINVAL;
}

int oo_or_remove(oo_or_tables* t, int af, const void* laddr, uint16_t lport,
                 const void* raddr, uint16_t rport, uint8_t proto, int32_t id)
{
  if( laddr == NULL || id < 0 || (uint32_t)id >= t->max_socks )
    return -EINVAL;
  if( af == 4 )
    ip4_remove(t, id, ld32(laddr), lport, raddr ? ld32(raddr) : 0, rport,
               proto);
  else if( af == 6 )
    ip6_remove(t, id, laddr, lport, raddr ? raddr : zero16, rport, proto);
  else
    return -EINVAL;
  return 0;
}

/* ci_ip4_netif_filter_lookup (netif_table.c:86-143) /
 * ci_ip6_netif_filter_lookup (netif_table_ip6.c:13-66). */
int oo_or_lookup(const oo_or_tables* t, int af, const void* laddr,
                 uint16_t lport, const void* raddr, uint16_t rport,
                 uint8_t proto)
{
  if( af == 4 ) {
    uint32_t la = ld32(laddr), ra = raddr ? ld32(raddr) : 0;
    uint32_t h1 = oo_or_hash1(t->ip4_mask, la, lport, ra, rport, proto);
    uint32_t h2 = 0, first = h1;
    while( 1 ) {
      uint32_t st = t->ip4_id_state[h1];
      if( OCCUPIED(st) ) {
        const oo_gpu_rx_sock* s = &t->socks[st & ID_MASK];
        if( la == t->ip4_laddr[h1] && lport == t->ip4_lport[h1] &&
            ra == s->raddr_be32 && rport == s->rport_be16 && proto == s->protocol )
          return (int)h1;
      }
      if( (st & ST_MASK) == ST_EMPTY )
        break;
      if( h1 == first )
        h2 = oo_or_hash2(la, lport, ra, rport, proto);
      h1 = (h1 + h2) & t->ip4_mask;
      if( h1 == first )
        return -ELOOP;
    }
    return -ENOENT;
  }
  if( af == 6 ) {
    const uint8_t* ra = raddr ? raddr : zero16;
    uint32_t lx = oo_or_addr_xor(laddr), rx = oo_or_addr_xor(ra);
    uint32_t h1 = oo_or_hash1(t->ip6_mask, lx, lport, rx, rport, proto);
    uint32_t h2 = 0, first = h1;
    while( 1 ) {
      int32_t id = t->ip6[h1].id;
      if( id >= 0 ) {
        const oo_gpu_rx_sock* s = &t->socks[id];
        if( lport == s->lport_be16 && rport == s->rport_be16 &&
            proto == s->protocol &&
            memcmp(laddr, t->ip6[h1].laddr, 16) == 0 &&
            memcmp(ra, s->raddr6, 16) == 0 )
          return (int)h1;
      }
      if( id == ID6_EMPTY )
        break;
      if( h1 == first )
        h2 = oo_or_hash2(lx, lport, rx, rport, proto);
      h1 = (h1 + h2) & t->ip6_mask;
      if( h1 == first )
        return -ELOOP;
    }
    return -ENOENT;
  }
  return -EINVAL;
}

int oo_or_slot(const oo_or_tables* t, int af, uint32_t slot,
               uint32_t* id_state, int32_t* route_count, uint16_t* lport)
{
  if( af == 4 ) {
    if( slot > t->ip4_mask )
      return -EINVAL;
    *id_state = t->ip4_id_state[slot];
    *route_count = t->ip4_route[slot];
    *lport = t->ip4_lport[slot];
    return 0;
  }
  if( af == 6 ) {
    if( slot > t->ip6_mask )
      return -EINVAL;
    *id_state = (uint32_t)t->ip6[slot].id;
    *route_count = t->ip6[slot].route_count;
    *lport = 0;
    return 0;
  }
  return -EINVAL;
}

/* Every slot that differs from its initial state, as rows of six int64
 * {af, slot, a, b, c, d}: IPv4 {id_state, laddr, route_count, lport}, IPv6
 * {id, route_count, laddr[0..7], laddr[8..15]} (little-endian halves) -- the
 * dump format of the table fixtures (tests/golden/make_table_golden.py).
 * Returns the number of rows (rows may be NULL to count). */
uint32_t oo_or_dump(const oo_or_tables* t, int64_t* rows, uint32_t cap)
{
  uint32_t i, n = 0;
  for( i = 0; i <= t->ip4_mask; ++i )
    if( t->ip4_id_state[i] != ST_EMPTY || t->ip4_laddr[i] || t->ip4_route[i] ||
        t->ip4_lport[i] ) {
      if( rows && n < cap ) {
        int64_t* r = rows + 6 * (size_t)n;
        r[0] = 4; r[1] = i; r[2] = t->ip4_id_state[i]; r[3] = t->ip4_laddr[i];
        r[4] = t->ip4_route[i]; r[5] = t->ip4_lport[i];
      }
      ++n;
    }
  for( i = 0; i <= t->ip6_mask; ++i ) {
    const ip6e_t* e = &t->ip6[i];
    int64_t lo, hi;
    memcpy(&lo, e->laddr, 8);
    memcpy(&hi, e->laddr + 8, 8);
    if( e->id != ID6_EMPTY || e->route_count || lo || hi ) {
      if( rows && n < cap ) {
        int64_t* r = rows + 6 * (size_t)n;
        r[0] = 6; r[1] = i; r[2] = e->id; r[3] = e->route_count; r[4] = lo; r[5] = hi;
      }
      ++n;
    }
  }
  return n;
}

/* ------------------------------------------------------------------ */
/* Demux walks: count every match of one stage, remember the first.     */

typedef struct { int32_t first; int n; } match_t;

/* ci_sock_intf_check (netif_table.h:30-36) behind the
 * rx_bind2dev_ifindex == CI_IFID_BAD test (netif_table.c:225-228). */
static inline int bind2dev_ok(const oo_or_tables* t, const oo_gpu_rx_sock* s,
                              int intf_i, int vlan)
{
  unsigned hw;
  if( !(s->flags & OO_GPU_RX_SOCK_BIND2DEV) )
    return 1;
  hw = (intf_i >= 0 && intf_i < OO_GPU_RX_MAX_INTF) ? t->hwport[intf_i] : 0xffu;
  return hw < 64 && (s->bind2dev_hwports & (1ull << hw)) != 0 &&
         s->bind2dev_vlan == vlan;
}

/* ci_netif_filter_for_each_match (netif_table.c:234-319).  stop: the
 * callback ends the walk at the first match (handle_entry, :225-229) -- TCP's
 * ci_tcp_rx_deliver_to_conn / _to_listen always return 1 (tcp_rx.c:
 * 4644-4657); otherwise (UDP, whose ci_udp_rx_deliver continues past a
 * multicast destination or a socket that drops, udp_rx.c:194-228) every
 * match is counted and the walk runs to its end. */
static match_t walk4(const oo_or_tables* t, uint32_t la, uint32_t lp,
                     uint32_t ra, uint32_t rp, uint32_t proto, int intf_i,
                     int vlan, int stop)
{
  match_t m = { -1, 0 };
  uint32_t h1 = oo_or_hash1(t->ip4_mask, la, lp, ra, rp, proto);
  uint32_t h2 = 0, first = h1, st = t->ip4_id_state[h1];
  int check_lport = 0;
  while( 1 ) {
    if( (check_lport && OCCUPIED(st)) ||
        (!check_lport && (st & ST_MASK) == ST_PREFERRED) ) {
      const oo_gpu_rx_sock* s = &t->socks[st & ID_MASK];
      if( la == t->ip4_laddr[h1] &&
          (!check_lport || lp == t->ip4_lport[h1]) &&
          ra == s->raddr_be32 && rp == s->rport_be16 && proto == s->protocol &&
          bind2dev_ok(t, s, intf_i, vlan) ) {
        if( m.n++ == 0 )
          m.first = (int32_t)(st & ID_MASK);
        if( stop )
          break;
      }
    }
    if( (st & ST_MASK) == ST_EMPTY )
      break;
    if( h1 == first )
      h2 = oo_or_hash2(la, lp, ra, rp, proto);
    h1 = (h1 + h2) & t->ip4_mask;
    if( h1 == first )
      break;
    st = t->ip4_id_state[h1];
    check_lport = 1;
  }
  return m;
}

/* ci_netif_filter_for_each_match_ip6 (netif_table_ip6.c:110-189); stop as
 * in walk4. */
static match_t walk6(const oo_or_tables* t, const uint8_t* la, uint32_t lp,
                     const uint8_t* ra /* NULL = [::] */, uint32_t rp,
                     uint32_t proto, int intf_i, int vlan, int stop)
{
  match_t m = { -1, 0 };
  uint32_t lx = oo_or_addr_xor(la), rx = oo_or_addr_xor(ra);
  uint32_t h1 = oo_or_hash1(t->ip6_mask, lx, lp, rx, rp, proto);
  uint32_t h2 = 0, first = h1;
  while( 1 ) {
    int32_t id = t->ip6[h1].id;
    if( id >= 0 ) {
      const oo_gpu_rx_sock* s = &t->socks[id];
      if( memcmp(la, t->ip6[h1].laddr, 16) == 0 && lp == s->lport_be16 &&
          proto == s->protocol &&
          ((ra == NULL && !(s->flags & OO_GPU_RX_SOCK_CONNECTED)) ||
           (ra != NULL && memcmp(ra, s->raddr6, 16) == 0 && rp == s->rport_be16)) &&
          bind2dev_ok(t, s, intf_i, vlan) ) {
        if( m.n++ == 0 )
          m.first = id;
        if( stop )
          break;
      }
    }
    else if( id == ID6_EMPTY )
      break;
    if( h1 == first )
      h2 = oo_or_hash2(lx, lp, rx, rp, proto);
    h1 = (h1 + h2) & t->ip6_mask;
    if( h1 == first )
      break;
  }
  return m;
}

/* One IPv4 lookup stage from outside (tests/poll_util.py restates the
 * future rule of udp_internal.h:41-103 over the stages' match counts). */
int oo_or_walk4(const oo_or_tables* t, uint32_t la, uint32_t lp, uint32_t ra, uint32_t rp,
                uint32_t proto, int intf_i, int vlan, int stop, int32_t* first)
{
  match_t m = walk4(t, la, lp, ra, rp, proto, intf_i, vlan, stop);
  if( first )
    *first = m.first;
  return m.n;
}

/* ------------------------------------------------------------------ */
/* IP options walk: ci_ip_options_parse (netif_event.c:135-185).  Option
 * lengths are read through plain (signed on x86) char, so a length byte
 * >= 128 is negative and fails the >= IPOPT_MINOFF(4) test. */
static int ip_options_bad(frame_t f, int opt, int end)
{
  int err = 0;
  while( rd8(f, opt) != 0 /* IPOPT_EOL */ && opt < end && !err ) {
    switch( rd8(f, opt) ) {
    case 1:   /* IPOPT_NOP */
      ++opt;
      break;
    case 7:   /* IPOPT_RR */
    case 68:  /* IPOPT_TS */
    case 130: /* IPOPT_SEC */
    case 136: /* IPOPT_SID */ {
      int l = (int)(int8_t)rd8(f, opt + 1);
      if( l < 4 || l > end - opt )
        err = 1;
      else
        opt += l;
      break;
    }
    default:  /* IPOPT_SSRR(137), IPOPT_LSRR(131), anything else */
      err = 1;
      break;
    }
  }
  return err;
}

/* ------------------------------------------------------------------ */
/* One frame. */

void oo_or_rx_one(const oo_or_tables* t, const uint8_t* frame, int len,
                  int intf_i, oo_gpu_rx_result* r)
{
  frame_t f = { frame, len };
  int pre_l3, l3, l4, ip_len = 0, ip_paylen, ihl4 = 0, is6, vlan;
  unsigned proto, et;

  memset(r, 0, sizeof(*r));
  r->sock = -1;

  /* ci_parse_rx_vlan (netif_event.c:116-132). */
  if( be16(f, 12) != 0x8100 ) {
    pre_l3 = 14;
    vlan = 0;
  }
  else {
    pre_l3 = 18;
    vlan = be16(f, 14) & 0xfff;
    r->flags |= OO_RX_F_VLAN;
  }
  r->vlan = (uint16_t)vlan;
  l3 = pre_l3;

  /* handle_rx_csum_bad (netif_event.c:1030-1082). */
  if( len < pre_l3 + 20 ) {
    r->reason = OO_RX_R_SHORT_L2;
    return;
  }
  et = be16(f, pre_l3 - 2);
  if( et == 0x0800 ) {
    is6 = 0;
    ip_len = (int)be16(f, l3 + 2);
    ihl4 = (int)(rd8(f, l3) & 0xf) * 4;
    ip_paylen = ip_len - ihl4;
    proto = rd8(f, l3 + 9);
    r->proto = (uint8_t)proto;
    r->ip_paylen = (uint16_t)ip_paylen;
    if( ip_paylen <= 0 || len < pre_l3 + ip_len ) {
      r->reason = OO_RX_R_IP4_LEN;
      return;
    }
    if( !oo_or_ip4_hdr_ok(frame + l3, len - pre_l3) ) {
      r->reason = OO_RX_R_IP4_CSUM;
      return;
    }
    l4 = l3 + ihl4;
  }
  else if( et == 0x86dd ) {
    is6 = 1;
    r->flags |= OO_RX_F_IP6;
    ip_paylen = (int)be16(f, l3 + 4);
    proto = rd8(f, l3 + 6);
    r->proto = (uint8_t)proto;
    r->ip_paylen = (uint16_t)ip_paylen;
    if( ip_paylen <= 0 || len < pre_l3 + 40 + ip_paylen ) {
      r->reason = OO_RX_R_IP6_LEN;
      return;
    }
    l4 = l3 + 40;
  }
  else {
    r->reason = OO_RX_R_NOT_IP;
    return;
  }

  /* L4 gates + checksum (netif_event.c:1084-1127). */
  if( proto == 6 ) {
    int hlen;
    if( ip_paylen < 20 ) {
      r->reason = OO_RX_R_TCP_SHORT;
      return;
    }
    /* ci_tcp_csum_correct (netif_event.c:97-113). */
    hlen = (int)((rd8(f, l4 + 12) & 0xf0u) >> 2);
    if( hlen < 20 || ip_paylen < hlen ||
        !(is6 ? oo_or_tcp6_ok(frame + l3, frame + l4, frame + l4 + hlen,
                              (size_t)(ip_paylen - hlen))
              : oo_or_tcp4_ok(frame + l3, frame + l4, frame + l4 + hlen,
                              (size_t)(ip_paylen - hlen))) ) {
      r->reason = OO_RX_R_TCP_CSUM;
      return;
    }
  }
  else if( proto == 17 ) {
    /* pkt->pf.udp.pay_len is a u32 (ip_shared_types.h:245). */
    uint32_t udp_pay = (uint32_t)be16(f, l4 + 4) - 8u;
    unsigned check;
    if( ip_paylen < 8 ) {
      r->reason = OO_RX_R_UDP_SHORT;
      return;
    }
    /* ci_udp_csum_correct (udp_rx.c:101-121): a 64-bit compare against
     * ipx_hdr_tot_len - CI_IPX_IHL, i.e. ip_paylen (ipvx.h:309-377). */
    if( (uint64_t)udp_pay + 8u > (uint64_t)(uint32_t)ip_paylen ) {
      r->reason = OO_RX_R_UDP_CSUM;
      return;
    }
    check = rd16n(f, l4 + 6);
    if( !(check == 0 && !is6) &&
        !(is6 ? oo_or_udp6_ok(frame + l3, frame + l4, frame + l4 + 8, udp_pay)
              : oo_or_udp4_ok(frame + l3, frame + l4, frame + l4 + 8, udp_pay)) ) {
      r->reason = OO_RX_R_UDP_CSUM;
      return;
    }
  }
  else {
    r->reason = OO_RX_R_PROTO_OTHER;
    return;
  }

  /* Handled: __handle_rx_pkt -> ci_parse_rx_vlan -> handle_rx_pkt
   * (netif_event.c:688-697, 250-451). */
  r->flags |= OO_RX_F_CSUM_OK;
  /* The TCP timestamp-option fast layout that ci_tcp_rx_deliver_to_conn
   * tests before its full option parser (tcp_rx.c:4537-4543): the header
   * length byte exactly (20 + 12) << 2, the first options word
   * CI_TCP_TSO_WORD = NOP NOP TIMESTAMP 10 (ip_shared_types.h:2742). */
  if( proto == 6 && rd8(f, l4 + 12) == 0x80u && rd32n(f, l4 + 20) == 0x0a080101u )
    r->flags |= OO_RX_F_TSO;
  r->l4_off = (uint16_t)l4;
  r->sport_be = (uint16_t)rd16n(f, l4);
  r->dport_be = (uint16_t)rd16n(f, l4 + 2);
  if( is6 ) {
    r->saddr_be = oo_or_addr_xor(frame + l3 + 8);
    r->daddr_be = oo_or_addr_xor(frame + l3 + 24);
  }
  else {
    unsigned frag = be16(f, l3 + 6);
    int not_fast;
    r->saddr_be = rd32n(f, l3 + 12);
    r->daddr_be = rd32n(f, l3 + 16);
    /* netif_event.c:293-303: MF/offset, tot_len vs frame, then options. */
    not_fast = (frag & 0x3fffu) != 0 || ip_len > len - pre_l3;
    if( not_fast ) {
      r->reason = OO_RX_R_IP4_FRAG;
      return;
    }
    if( ihl4 > 20 && ip_options_bad(f, l3 + 20, l3 + ihl4) ) {
      r->reason = OO_RX_R_IP4_OPTS_BAD;
      return;
    }
    /* ci_tcp_handle_rx frag test (tcp_rx.c:4696-4699): only 0 or DF. */
    if( proto == 6 && frag != 0x4000u && frag != 0 ) {
      r->reason = OO_RX_R_TCP_SCATTERED;
      return;
    }
  }

  /* Demux: UDP udp_rx.c:271-306; TCP tcp_rx.c:4786-4835. */
  {
    match_t m[3];
    int nst = proto == 6 ? 3 : 2, s;
    uint32_t sport = r->sport_be, dport = r->dport_be;
    if( is6 ) {
      const uint8_t* sa = frame + l3 + 8;
      const uint8_t* da = frame + l3 + 24;
      r->hash3 = oo_or_hash3(oo_or_addr_xor(da), dport, oo_or_addr_xor(sa),
                             sport, proto);
      m[0] = walk6(t, da, dport, sa, sport, proto, intf_i, vlan, nst == 3);
      m[1] = walk6(t, da, dport, NULL, 0, proto, intf_i, vlan, nst == 3);
      if( nst == 3 )
        m[2] = walk6(t, zero16, dport, NULL, 0, proto, intf_i, vlan, 1);
    }
    else {
      uint32_t sa = r->saddr_be, da = r->daddr_be;
      r->hash3 = oo_or_hash3(da, dport, sa, sport, proto);
      m[0] = walk4(t, da, dport, sa, sport, proto, intf_i, vlan, nst == 3);
      m[1] = walk4(t, da, dport, 0, 0, proto, intf_i, vlan, nst == 3);
      if( nst == 3 )
        m[2] = walk4(t, 0, dport, 0, 0, proto, intf_i, vlan, 1);
    }
    if( proto == 17 ) {
      /* ci_udp_rx_deliver's multi-destination test reads the IPv4 view of
       * the L3 header, ip_daddr_be32 = bytes 16..19 (udp_rx.c:157-159). */
      uint32_t d = rd32n(f, l3 + 16);
      if( (d & 0xf0u) == 0xe0u || d == 0xffffffffu )
        r->flags |= OO_RX_F_MCAST;
    }
    r->reason = OO_RX_R_NO_MATCH;
    for( s = 0; s < nst; ++s )
      if( m[s].n > 0 ) {
        r->reason = OO_RX_R_DELIVER;
        r->stage = (uint8_t)(s + 1);
        r->sock = m[s].first;
        r->nmatch = (uint16_t)m[s].n;
        if( m[s].n > 1 )
          r->flags |= OO_RX_F_MULTI;
        /* The future rule's union (udp_internal.h:41-52, :86-97): after a
         * single stage-1 match ci_udp_handle_rx_pre_future still walks
         * stage 2, and any match there gives the future up. */
        if( proto == 17 && !is6 && s == 0 && m[0].n == 1 && m[1].n > 0 )
          r->flags |= OO_RX_F_UDP_S2;
        break;
      }
  }
}

/* ------------------------------------------------------------------ */
/* Batch over host threads. */

typedef struct {
  const oo_or_tables* t;
  const uint8_t* frames;
  uint64_t frames_bytes;
  const oo_gpu_pkt_desc* d;
  oo_gpu_rx_result* out;
  uint32_t lo, hi;
} shard_t;

static void* run_shard(void* arg)
{
  shard_t* s = arg;
  uint32_t i;
  for( i = s->lo; i < s->hi; ++i ) {
    /* A descriptor outside the frame buffer is an empty frame (the batch
     * boundary's rule; the overflow-safe form of off + len <= bytes). */
    const uint64_t off = s->d[i].frame_off;
    if( off <= s->frames_bytes && (uint64_t)s->d[i].len <= s->frames_bytes - off )
      oo_or_rx_one(s->t, s->frames + off, s->d[i].len, s->d[i].intf_i, &s->out[i]);
    else
      oo_or_rx_one(s->t, s->frames, 0, s->d[i].intf_i, &s->out[i]);
  }
  return NULL;
}

void oo_or_rx_batch(const oo_or_tables* t, const uint8_t* frames,
                    uint64_t frames_bytes, const oo_gpu_pkt_desc* d, uint32_t n,
                    oo_gpu_rx_result* out, int nthreads)
{
  pthread_t th[256];
  shard_t sh[256];
  int k;
  if( nthreads < 1 )
    nthreads = 1;
  if( nthreads > 256 )
    nthreads = 256;
  for( k = 0; k < nthreads; ++k ) {
    sh[k].t = t; sh[k].frames = frames; sh[k].frames_bytes = frames_bytes;
    sh[k].d = d; sh[k].out = out;
    sh[k].lo = (uint32_t)((uint64_t)n * k / nthreads);
    sh[k].hi = (uint32_t)((uint64_t)n * (k + 1) / nthreads);
  }
  if( nthreads == 1 ) {
    run_shard(&sh[0]);
    return;
  }
  for( k = 0; k < nthreads; ++k )
    pthread_create(&th[k], NULL, run_shard, &sh[k]);
  for( k = 0; k < nthreads; ++k )
    pthread_join(th[k], NULL);
}

/* ------------------------------------------------------------------ */
/* TX checksum fill.                            */

/* The fill value of an exact word sum S != 0: ip_proto_csum64_finish
 * (checksum.c:162-174) folds with end-around carry and complements, so a
 * sum that is a non-zero multiple of 0xffff gives 0. */
static inline uint32_t fill_of(uint64_t s)
{ return (~fold16(s)) & 0xffffu; }

static inline void st16n(uint8_t* p, uint32_t v)
{ p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); }

/* oo_pkt_calc_checksums (src/lib/transport/ip/pkt_checksum.c:20-102) as
 * calc_csum_if_needed (netif_tx.c:24-40) calls it: only for TCP or UDP
 * (ipx_hdr_protocol); the IPv4 header checksum (ef_ip_checksum,
 * checksum.c:185-212: the 4*IHL header bytes without the check field), then
 * the L4 check field over the rest of the frame:
 *   UDP (ef_udp_checksum{,_ip6}, checksum.c:225-250): not for an IPv4
 *     fragment (ci_ipx_is_frag: frag_off bits other than DF, ipvx.h:474-488);
 *     pseudo-header + header words 0..2 + payload from udp+8; 0 -> 0xffff;
 *   TCP (ef_tcp_checksum{,_ip6}, checksum.c:260-296): pseudo-header with
 *     (u16)(tot_len - 4*IHL) (IPv4) or payload_len (IPv6), the 4*doff
 *     header bytes, + 0xffff - check, payload from tcp+4*doff.
 * The VLAN tag is parsed as on RX (ci_parse_rx_vlan).  The reference
 * asserts the headers lie in the frame; here a frame whose headers do not
 * fit, or with IHL < 5 or TCP doff < 5, is left untouched. */
void oo_or_tx_fill_one(uint8_t* fr, int len)
{
  frame_t f = { fr, len };
  int l3 = 14, l4, af6, ihl4 = 40;
  unsigned proto;
  uint64_t pseudo;
  if( len < 14 )
    return;
  if( be16(f, 12) == 0x8100u )
    l3 = 18;
  switch( be16(f, l3 - 2) ) {
  case 0x0800u: af6 = 0; break;
  case 0x86ddu: af6 = 1; break;
  default: return;
  }
  if( !af6 ) {
    if( len < l3 + 20 )
      return;
    ihl4 = (fr[l3] & 0xf) * 4;
    if( ihl4 < 20 || len < l3 + ihl4 )
      return;
    proto = fr[l3 + 9];
  }
  else {
    if( len < l3 + 40 )
      return;
    proto = fr[l3 + 6];
  }
  if( proto != 6u && proto != 17u )
    return;
  l4 = l3 + ihl4;
  if( !af6 )  /* ip_hdr_csum32_finish: no 0 -> 0xffff substitution */
    st16n(fr + l3 + 10, fill_of(sum16(fr + l3, (size_t)ihl4) - rd16n(f, l3 + 10)));
  if( proto == 17u ) {
    uint32_t v;
    if( !af6 && (be16(f, l3 + 6) & ~0x4000u) )
      return;
    if( len < l4 + 8 )
      return;
    pseudo = af6 ? sum16(fr + l3 + 8, 32) : ip4_addr_sum(fr + l3);
    pseudo += 0x1100u + rd16n(f, l4 + 4);
    v = fill_of(pseudo + sum16(fr + l4, 6) + sum16(fr + l4 + 8, (size_t)(len - l4 - 8)));
    st16n(fr + l4 + 6, v ? v : 0xffffu);
  }
  else {
    int hl4;
    if( len < l4 + 20 )
      return;
    hl4 = (fr[l4 + 12] >> 4) * 4;
    if( hl4 < 20 || len < l4 + hl4 )
      return;
    if( af6 ) {
      pseudo = sum16(fr + l3 + 8, 32) + rd16n(f, l3 + 4);
    }
    else {
      unsigned pl = (be16(f, l3 + 2) - (unsigned)ihl4) & 0xffffu;
      pseudo = ip4_addr_sum(fr + l3) + (((pl & 0xffu) << 8) | (pl >> 8));
    }
    pseudo += 0x0600u;
    st16n(fr + l4 + 16, fill_of(pseudo + sum16(fr + l4, (size_t)hl4) +
                                (0xffffu - rd16n(f, l4 + 16)) +
                                sum16(fr + l4 + hl4, (size_t)(len - l4 - hl4))));
  }
}

/* efxdp_ef_eventq_poll's RX branch (src/lib/ciul/efxdp_vi.c:316-356) and
 * the event -> packet step of ci_netif_poll_evq (netif_event.c:1715-1736),
 * for n entries from consumer index cons: entry (cons + i) & mask gives
 * rq_id = addr / 2048, ofs = addr & 2047 (the frame at UMEM + addr, its
 * buffer being UMEM + rq_id * 2048), rx.len = the low 16 bits of len
 * (ef_event's 16-bit field, ef_vi.h:154), then the per-packet path on the
 * ring's interface.  An entry outside the UMEM is an empty frame (the
 * batch boundary's rule, not the reference's: it would read wild memory). */
void oo_or_xdp_batch(const oo_or_tables* t, const uint8_t* umem,
                     uint64_t umem_bytes, const oo_gpu_xdp_desc* ring,
                     uint32_t mask, uint32_t cons, uint32_t n, int intf_i,
                     oo_gpu_rx_result* out)
{
  uint32_t i;
  for( i = 0; i < n; ++i ) {
    const oo_gpu_xdp_desc* e = &ring[(cons + i) & mask];
    const uint64_t rq_id = e->addr / 2048u, ofs = e->addr & 2047u;
    const int len = (int)(e->len & 0xffffu);
    const uint64_t at = rq_id * 2048u + ofs;
    if( at <= umem_bytes && (uint64_t)len <= umem_bytes - at )
      oo_or_rx_one(t, umem + at, len, intf_i, &out[i]);
    else
      oo_or_rx_one(t, umem, 0, intf_i, &out[i]);
  }
}

void oo_or_tx_fill_batch(uint8_t* frames, uint64_t frames_bytes,
                         const oo_gpu_pkt_desc* d, uint32_t n)
{
  uint32_t i;
  for( i = 0; i < n; ++i ) {
    uint64_t off = d[i].frame_off;
    if( off <= frames_bytes && (uint64_t)d[i].len <= frames_bytes - off )
      oo_or_tx_fill_one(frames + off, d[i].len);
  }
}
