/* SPDX-License-Identifier: BSD-2-Clause */
/*
 * oo_pktgen.c -- seeded synthetic frame generator (see oo_pktgen.h).
 *
 * Workloads follow SURVEY.md §8(d):
 *  config 2: 1514 B IPv4/UDP to 512 unconnected sockets 10.0.0.1:6000+k,
 *            sport 32768..60999, saddr 10.1.x.y; 1% corrupted L4 checksum,
 *            0.5% UDP checksum 0, 0.5% unbound dport.
 *  config 3: the same at 64 B (22-byte payload).
 *  config 4: IPv4/TCP, log-uniform 64..9014 B, 20% with IP options
 *            (NOP/RR/TS/SEC/SID; 2% LSRR), TCP doff 5..15, 4096 connected
 *            sockets + 32 laddr-specific + 32 wildcard listeners (all three
 *            lookup stages), 5% unmatched, 1% bad checksum.
 *  config 5: IMIX 64:594:1518 (7:4:1), 70% TCP / 30% UDP, 80% IPv4 / 20%
 *            IPv6 over the union of the worlds above plus IPv6 sockets.
 */
#include "oo_pktgen.h"

#include <math.h>
#include <pthread.h>
#include <string.h>

/* ------------------------------------------------------------------ */

static inline uint64_t splitmix64(uint64_t* s)
{
  uint64_t z = (*s += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

static inline uint64_t pkt_state(uint64_t seed, uint64_t i)
{
  uint64_t s = seed ^ (i * 0xd1b54a32d192ed03ull);
  (void)splitmix64(&s);
  return s;
}

static inline void put16(uint8_t* p, unsigned v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
static inline uint16_t htons_(unsigned v) { return (uint16_t)(((v & 0xff) << 8) | ((v >> 8) & 0xff)); }

uint64_t oo_pg_default_seed(int config)
{
  return 0x4F4E4C4400000000ull | (uint64_t)(config & 0xff);
}

/* ------------------------------------------------------------------ */
/* The socket world. */

#define N_UDP4      512
#define N_TCP4_CONN 4096
#define N_TCP4_LIS  32
#define N_TCP4_WLD  32
#define N_UDP6      256
#define N_TCP6_CONN 1024
#define N_TCP6_LIS  8
#define N_TCP6_WLD  8

static const uint8_t LADDR4[4] = { 10, 0, 0, 1 };
static const uint8_t LADDR6[16] = { 0xfd, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1 };

static void tcp4_peer(int k, uint8_t* a) { a[0] = 10; a[1] = 2; a[2] = (uint8_t)(k >> 8); a[3] = (uint8_t)k; }
static void tcp6_peer(int k, uint8_t* a)
{ memset(a, 0, 16); a[0] = 0xfd; a[3] = 2; a[14] = (uint8_t)(k >> 8); a[15] = (uint8_t)k; }

/* Socket id bases. */
enum {
  SB_UDP4 = 0,
  SB_TCP4_CONN = SB_UDP4 + N_UDP4,
  SB_TCP4_LIS = SB_TCP4_CONN + N_TCP4_CONN,
  SB_TCP4_WLD = SB_TCP4_LIS + N_TCP4_LIS,
  SB_UDP6 = SB_TCP4_WLD + N_TCP4_WLD,
  SB_TCP6_CONN = SB_UDP6 + N_UDP6,
  SB_TCP6_LIS = SB_TCP6_CONN + N_TCP6_CONN,
  SB_TCP6_WLD = SB_TCP6_LIS + N_TCP6_LIS,
  SB_END = SB_TCP6_WLD + N_TCP6_WLD
};

static int world_has(int config, int part)
{
  switch( part ) {
  case 0: return config == 2 || config == 3 || config == 5;   /* udp4 */
  case 1: return config == 4 || config == 5;                  /* tcp4 */
  case 2: return config == 5;                                 /* v6   */
  }
  return 0;
}

static int add(oo_pg_filter* f, int nf, int max, int sock, int af, int proto,
               const uint8_t* la, unsigned lport, const uint8_t* ra,
               unsigned rport)
{
  if( nf >= max )
    return nf;
  memset(&f[nf], 0, sizeof(f[nf]));
  f[nf].sock = sock;
  f[nf].af = (uint8_t)af;
  f[nf].proto = (uint8_t)proto;
  f[nf].lport_be = htons_(lport);
  f[nf].rport_be = htons_(rport);
  memcpy(f[nf].laddr, la, af == 4 ? 4 : 16);
  if( ra == NULL )
    f[nf].raddr_any = 1;
  else
    memcpy(f[nf].raddr, ra, af == 4 ? 4 : 16);
  return nf + 1;
}

int oo_pg_world(int config, oo_pg_filter* f, int max, oo_gpu_rx_sock* socks,
                int max_socks, int* n_socks)
{
  int nf = 0, k;
  uint8_t a[16];
  static const uint8_t any[16];
  if( config < 2 || config > 5 || max_socks < SB_END )
    return -1;
  memset(socks, 0, sizeof(*socks) * SB_END);
  if( world_has(config, 0) )
    for( k = 0; k < N_UDP4; ++k ) {
      oo_gpu_rx_sock* s = &socks[SB_UDP4 + k];
      s->protocol = 17;
      s->lport_be16 = htons_(6000 + k);
      nf = add(f, nf, max, SB_UDP4 + k, 4, 17, LADDR4, 6000 + k, NULL, 0);
    }
  if( world_has(config, 1) ) {
    for( k = 0; k < N_TCP4_CONN; ++k ) {
      oo_gpu_rx_sock* s = &socks[SB_TCP4_CONN + k];
      tcp4_peer(k, a);
      memcpy(&s->raddr_be32, a, 4);
      s->rport_be16 = htons_(33000 + k);
      s->lport_be16 = htons_(8000 + (k & 63));
      s->protocol = 6;
      s->flags = OO_GPU_RX_SOCK_CONNECTED;
      nf = add(f, nf, max, SB_TCP4_CONN + k, 4, 6, LADDR4, 8000 + (k & 63), a, 33000 + k);
    }
    for( k = 0; k < N_TCP4_LIS; ++k ) {
      oo_gpu_rx_sock* s = &socks[SB_TCP4_LIS + k];
      s->protocol = 6;
      s->lport_be16 = htons_(9000 + k);
      nf = add(f, nf, max, SB_TCP4_LIS + k, 4, 6, LADDR4, 9000 + k, NULL, 0);
    }
    for( k = 0; k < N_TCP4_WLD; ++k ) {
      oo_gpu_rx_sock* s = &socks[SB_TCP4_WLD + k];
      s->protocol = 6;
      s->lport_be16 = htons_(9100 + k);
      nf = add(f, nf, max, SB_TCP4_WLD + k, 4, 6, any, 9100 + k, NULL, 0);
    }
  }
  if( world_has(config, 2) ) {
    for( k = 0; k < N_UDP6; ++k ) {
      oo_gpu_rx_sock* s = &socks[SB_UDP6 + k];
      s->protocol = 17;
      s->lport_be16 = htons_(7000 + k);
      nf = add(f, nf, max, SB_UDP6 + k, 6, 17, LADDR6, 7000 + k, NULL, 0);
    }
    for( k = 0; k < N_TCP6_CONN; ++k ) {
      oo_gpu_rx_sock* s = &socks[SB_TCP6_CONN + k];
      tcp6_peer(k, a);
      memcpy(s->raddr6, a, 16);
      s->rport_be16 = htons_(34000 + k);
      s->lport_be16 = htons_(8500 + (k & 63));
      s->protocol = 6;
      s->flags = OO_GPU_RX_SOCK_CONNECTED;
      nf = add(f, nf, max, SB_TCP6_CONN + k, 6, 6, LADDR6, 8500 + (k & 63), a, 34000 + k);
    }
    for( k = 0; k < N_TCP6_LIS; ++k ) {
      oo_gpu_rx_sock* s = &socks[SB_TCP6_LIS + k];
      s->protocol = 6;
      s->lport_be16 = htons_(9200 + k);
      nf = add(f, nf, max, SB_TCP6_LIS + k, 6, 6, LADDR6, 9200 + k, NULL, 0);
    }
    for( k = 0; k < N_TCP6_WLD; ++k ) {
      oo_gpu_rx_sock* s = &socks[SB_TCP6_WLD + k];
      s->protocol = 6;
      s->lport_be16 = htons_(9300 + k);
      nf = add(f, nf, max, SB_TCP6_WLD + k, 6, 6, any, 9300 + k, NULL, 0);
    }
  }
  *n_socks = SB_END;
  return nf;
}

/* ------------------------------------------------------------------ */
/* Packet specification drawn from the per-packet RNG. */

typedef struct {
  uint32_t len;      /* frame length */
  int af;            /* 4 or 6 */
  int proto;         /* 6 or 17 */
  int ihl;           /* IPv4 IHL words (5..15) */
  int doff;          /* TCP data offset words */
  int opt_lsrr;      /* put an LSRR option (-> IP4_OPTS_BAD) */
  int bad_csum;      /* corrupt one L4 byte after the checksum */
  int zero_csum;     /* UDP checksum 0 */
  unsigned sport, dport;
  uint8_t saddr[16], daddr[16];
  uint64_t rng;      /* state for the payload bytes */
} spec_t;

static uint32_t imix_len(uint64_t r)
{
  unsigned k = (unsigned)(r % 12);
  return k < 7 ? 64u : k < 11 ? 594u : 1518u;
}

static void pick_tcp_dest(spec_t* s, uint64_t r, int af)
{
  unsigned u = (unsigned)(r % 100);
  unsigned k = (unsigned)((r >> 8) % (af == 4 ? N_TCP4_CONN : N_TCP6_CONN));
  if( u < 60 ) {          /* established: stage 1 */
    if( af == 4 ) { tcp4_peer((int)k, s->saddr); s->sport = 33000 + k; s->dport = 8000 + (k & 63); }
    else          { tcp6_peer((int)k, s->saddr); s->sport = 34000 + k; s->dport = 8500 + (k & 63); }
  }
  else if( u < 80 )       /* laddr-specific listener: stage 2 */
    s->dport = (af == 4 ? 9000u : 9200u) + (unsigned)((r >> 24) % (af == 4 ? N_TCP4_LIS : N_TCP6_LIS));
  else if( u < 95 )       /* wildcard listener: stage 3 */
    s->dport = (af == 4 ? 9100u : 9300u) + (unsigned)((r >> 24) % (af == 4 ? N_TCP4_WLD : N_TCP6_WLD));
  else                    /* nobody: NO_MATCH */
    s->dport = 20000 + (unsigned)((r >> 24) % 1000);
}

static void draw(int config, uint64_t seed, uint64_t i, spec_t* s)
{
  uint64_t st = pkt_state(seed, i);
  uint64_t r0 = splitmix64(&st), r1 = splitmix64(&st), r2 = splitmix64(&st);
  uint64_t r3 = splitmix64(&st);
  unsigned u = (unsigned)(r1 % 10000);
  memset(s, 0, sizeof(*s));
  s->af = 4;
  s->proto = 17;
  s->ihl = 5;
  s->doff = 5;
  /* default remote */
  s->saddr[0] = 10; s->saddr[1] = 1; s->saddr[2] = (uint8_t)(r2 >> 8); s->saddr[3] = (uint8_t)(r2 >> 16);
  memcpy(s->daddr, LADDR4, 4);
  s->sport = 32768 + (unsigned)((r2 >> 24) % 28232);

  if( config == 2 || config == 3 ) {
    s->len = config == 2 ? 1514 : 64;
    s->dport = 6000 + (unsigned)((r3) % N_UDP4);
    if( u < 100 ) s->bad_csum = 1;
    else if( u < 150 ) s->zero_csum = 1;
    else if( u < 200 ) s->dport = 6000 + N_UDP4 + (unsigned)(r3 % 1000);
  }
  else if( config == 4 ) {
    double x = (double)(r0 >> 11) * (1.0 / 9007199254740992.0);
    s->proto = 6;
    s->len = (uint32_t)(64.0 * exp2(x * log2(9014.0 / 64.0)));
    if( s->len < 64 ) s->len = 64;
    if( s->len > 9014 ) s->len = 9014;
    pick_tcp_dest(s, r3, 4);
    if( u < 100 ) s->bad_csum = 1;
    if( (r2 >> 40) % 100 < 20 ) s->ihl = 6 + (int)((r2 >> 48) % 10);
    if( u >= 100 && u < 300 ) { s->opt_lsrr = 1; if( s->ihl < 7 ) s->ihl = 7; }
    s->doff = 5 + (int)((r0 & 0xff) % 11);
  }
  else { /* config 5 */
    s->len = imix_len(r0);
    s->proto = (r1 >> 20) % 10 < 7 ? 6 : 17;
    s->af = (r1 >> 28) % 10 < 8 ? 4 : 6;
    if( u < 100 ) s->bad_csum = 1;
    if( s->af == 6 ) {
      memset(s->saddr, 0, 16);
      s->saddr[0] = 0xfd; s->saddr[3] = 1;
      memcpy(s->saddr + 8, &r2, 8);
      memcpy(s->daddr, LADDR6, 16);
    }
    if( s->proto == 6 ) {
      pick_tcp_dest(s, r3, s->af);
      s->doff = 5 + (int)((r0 >> 8) % 4);
    }
    else {
      unsigned n = s->af == 4 ? N_UDP4 : N_UDP6, base = s->af == 4 ? 6000 : 7000;
      s->dport = base + (unsigned)(r3 % n);
      if( u >= 100 && u < 200 ) s->dport = base + n + (unsigned)(r3 % 1000);
    }
  }
  /* Make the headers fit the frame. */
  {
    unsigned l3h = s->af == 4 ? (unsigned)s->ihl * 4 : 40;
    unsigned l4h = s->proto == 6 ? (unsigned)s->doff * 4 : 8;
    while( 14 + l3h + l4h > s->len ) {
      if( s->proto == 6 && s->doff > 5 ) { --s->doff; l4h -= 4; }
      else if( s->af == 4 && s->ihl > 5 && !(s->opt_lsrr && s->ihl <= 7) ) { --s->ihl; l3h -= 4; }
      else { s->len = 14 + l3h + l4h; break; }
    }
  }
  s->rng = st;
}

/* ------------------------------------------------------------------ */
/* RFC 1071 fill (pkt_checksum.c:20-102 semantics). */

static uint32_t sum_words(const uint8_t* p, uint32_t n)
{
  uint32_t s = 0, i = 0;
  for( ; i + 1 < n; i += 2 ) s += (uint32_t)p[i] << 8 | p[i + 1];
  if( i < n ) s += (uint32_t)p[i] << 8;
  return s;
}
static uint16_t csum_fin(uint64_t s)
{
  while( s >> 16 ) s = (s & 0xffff) + (s >> 16);
  return (uint16_t)~s;
}

uint32_t oo_pg_len(int config, uint64_t seed, uint64_t i)
{
  spec_t s;
  draw(config, seed, i, &s);
  return s.len;
}

uint64_t oo_pg_bytes(int config, uint64_t seed, uint64_t first, uint32_t n,
                     uint32_t align)
{
  uint64_t b = 0;
  uint32_t k;
  if( align == 0 ) align = 1;
  for( k = 0; k < n; ++k )
    b += (oo_pg_len(config, seed, first + k) + align - 1) / align * align;
  return b;
}

static void build(const spec_t* s, uint8_t* f)
{
  uint64_t st = s->rng;
  uint32_t l3 = 14, l3h, l4, l4h, l4len, k;
  uint8_t* ip = f + l3;
  /* Ethernet */
  f[0] = 0x02; f[1] = 0; f[2] = 0; f[3] = 0; f[4] = 0; f[5] = 1;
  f[6] = 0x02; f[7] = 0; f[8] = 0; f[9] = 0; f[10] = 0; f[11] = 2;
  put16(f + 12, s->af == 4 ? 0x0800 : 0x86dd);
  l3h = s->af == 4 ? (uint32_t)s->ihl * 4 : 40;
  l4 = l3 + l3h;
  l4h = s->proto == 6 ? (uint32_t)s->doff * 4 : 8;
  l4len = s->len - l4;
  /* payload first (random) */
  for( k = l4 + l4h; k < s->len; k += 8 ) {
    uint64_t r = splitmix64(&st);
    uint32_t m = s->len - k < 8 ? s->len - k : 8;
    memcpy(f + k, &r, m);
  }
  if( s->af == 4 ) {
    ip[0] = (uint8_t)(0x40 | s->ihl);
    ip[1] = 0;
    put16(ip + 2, s->len - l3);
    put16(ip + 4, (unsigned)(st & 0xffff));
    put16(ip + 6, 0x4000);  /* DF */
    ip[8] = 64;
    ip[9] = (uint8_t)s->proto;
    put16(ip + 10, 0);
    memcpy(ip + 12, s->saddr, 4);
    memcpy(ip + 16, s->daddr, 4);
    if( s->ihl > 5 ) {
      uint8_t* o = ip + 20;
      uint32_t ol = l3h - 20, p = 0;
      if( s->opt_lsrr ) {
        o[p++] = 131; o[p++] = 7; o[p++] = 4; o[p++] = 10; o[p++] = 0; o[p++] = 0; o[p++] = 9;
      }
      else {
        static const uint8_t kinds[4] = { 7, 68, 130, 136 };
        uint8_t kind = kinds[(st >> 20) & 3];
        unsigned ln = kind == 136 ? 4 : kind == 130 ? (ol >= 11 ? 11 : 4) : (ol >= 8 ? 8 : 4);
        o[p++] = 1;                       /* NOP */
        if( p + ln <= ol ) {
          o[p] = kind; o[p + 1] = (uint8_t)ln;
          for( k = 2; k < ln; ++k ) o[p + k] = (uint8_t)(k == 2 ? 4 : 0);
          p += ln;
        }
      }
      for( ; p < ol; ++p ) o[p] = (uint8_t)(p + 1 < ol ? 1 : 0);  /* NOPs, then EOL */
    }
    put16(ip + 10, csum_fin(sum_words(ip, l3h)));
  }
  else {
    ip[0] = 0x60; ip[1] = 0; ip[2] = 0; ip[3] = 0;
    put16(ip + 4, l4len);
    ip[6] = (uint8_t)s->proto;
    ip[7] = 64;
    memcpy(ip + 8, s->saddr, 16);
    memcpy(ip + 24, s->daddr, 16);
  }
  {
    uint8_t* l = f + l4;
    uint64_t ps;
    put16(l + 0, s->sport);
    put16(l + 2, s->dport);
    if( s->proto == 17 ) {
      put16(l + 4, l4len);
      put16(l + 6, 0);
    }
    else {
      uint64_t r = splitmix64(&st);
      memcpy(l + 4, &r, 8);                      /* seq, ack */
      l[12] = (uint8_t)(s->doff << 4);
      l[13] = 0x10;                              /* ACK */
      put16(l + 14, 65535);
      put16(l + 16, 0);
      put16(l + 18, 0);
      for( k = 20; k < l4h; ++k ) l[k] = 1;      /* NOP options */
      if( l4h >= 24 ) { l[20] = 2; l[21] = 4; put16(l + 22, 1460); }  /* MSS */
    }
    if( s->af == 4 )
      ps = sum_words(ip + 12, 8) + (uint32_t)s->proto + l4len;
    else
      ps = sum_words(ip + 8, 32) + (uint32_t)s->proto + l4len;
    if( !(s->proto == 17 && s->zero_csum) ) {
      uint16_t c = csum_fin(ps + sum_words(l, l4len));
      if( s->proto == 17 && c == 0 ) c = 0xffff;
      put16(l + (s->proto == 17 ? 6 : 16), c);
    }
    if( s->bad_csum ) {
      /* Flip one L4 byte that is not a port (ports steer the demux). */
      uint32_t at = l4len > 8 ? 4 + (uint32_t)((st >> 7) % (l4len - 4)) : 4;
      if( s->proto == 17 && at < 6 ) at = 6;
      l[at] ^= 0x5a;
      if( s->proto == 17 && at == 6 && l[6] == 0 && l[7] == 0 ) l[7] = 1;
    }
  }
}

typedef struct {
  int config; uint64_t seed, first; uint32_t lo, hi;
  uint8_t* buf; const oo_gpu_pkt_desc* desc;
} job_t;

static void* gen_job(void* a)
{
  job_t* j = a;
  uint32_t k;
  spec_t s;
  for( k = j->lo; k < j->hi; ++k ) {
    draw(j->config, j->seed, j->first + k, &s);
    build(&s, j->buf + j->desc[k].frame_off);
  }
  return NULL;
}

uint64_t oo_pg_gen(int config, uint64_t seed, uint64_t first, uint32_t n,
                   uint32_t align, uint8_t* buf, uint64_t cap,
                   oo_gpu_pkt_desc* desc, int nthreads)
{
  uint64_t off = 0;
  uint32_t k;
  if( align == 0 ) align = 1;
  for( k = 0; k < n; ++k ) {
    uint32_t len = oo_pg_len(config, seed, first + k);
    desc[k].frame_off = off;
    desc[k].len = (uint16_t)len;
    desc[k].intf_i = 0;
    desc[k].rsvd = 0;
    off += (len + align - 1) / align * align;
  }
  if( off > cap )
    return 0;
  if( nthreads < 1 ) nthreads = 1;
  if( nthreads > 64 ) nthreads = 64;
  {
    pthread_t th[64];
    job_t jobs[64];
    int t;
    for( t = 0; t < nthreads; ++t ) {
      jobs[t].config = config; jobs[t].seed = seed; jobs[t].first = first;
      jobs[t].lo = (uint32_t)((uint64_t)n * t / nthreads);
      jobs[t].hi = (uint32_t)((uint64_t)n * (t + 1) / nthreads);
      jobs[t].buf = buf; jobs[t].desc = desc;
    }
    if( nthreads == 1 )
      gen_job(&jobs[0]);
    else {
      for( t = 0; t < nthreads; ++t ) pthread_create(&th[t], NULL, gen_job, &jobs[t]);
      for( t = 0; t < nthreads; ++t ) pthread_join(th[t], NULL);
    }
  }
  return off;
}

/* Byte-balanced shard boundaries ("by cumulative bytes for
 * IMIX/jumbo"): rank r owns packets [firsts[r], firsts[r+1]), where firsts[r]
 * is the first packet whose packed bytes before it (at `align`) reach
 * r / world of the total.  Two threaded passes over the lengths. */
typedef struct {
  int config; uint64_t seed, lo, hi; uint32_t align; uint64_t bytes;
} split_job_t;

static void* split_job(void* a)
{
  split_job_t* j = a;
  uint64_t i, b = 0;
  for( i = j->lo; i < j->hi; ++i )
    b += (oo_pg_len(j->config, j->seed, i) + j->align - 1) / j->align * j->align;
  j->bytes = b;
  return NULL;
}

int oo_pg_split(int config, uint64_t seed, uint64_t n_total, int world, uint32_t align,
                uint64_t* firsts, int nthreads)
{
  enum { MAXT = 64 };
  pthread_t th[MAXT];
  split_job_t jobs[MAXT];
  uint64_t total = 0, before[MAXT + 1];
  int t, r;
  if( world < 1 || firsts == NULL ) return -1;
  if( align == 0 ) align = 1;
  if( nthreads < 1 ) nthreads = 1;
  if( nthreads > MAXT ) nthreads = MAXT;
  for( t = 0; t < nthreads; ++t ) {
    jobs[t].config = config; jobs[t].seed = seed; jobs[t].align = align;
    jobs[t].lo = n_total * (uint64_t)t / (uint64_t)nthreads;
    jobs[t].hi = n_total * (uint64_t)(t + 1) / (uint64_t)nthreads;
    pthread_create(&th[t], NULL, split_job, &jobs[t]);
  }
  for( t = 0; t < nthreads; ++t ) pthread_join(th[t], NULL);
  for( t = 0; t < nthreads; ++t ) {
    before[t] = total;
    total += jobs[t].bytes;
  }
  before[nthreads] = total;
  firsts[0] = 0;
  firsts[world] = n_total;
  for( r = 1; r < world; ++r ) {
    /* the first packet whose bytes-before reach ceil(total * r / world) */
    const uint64_t target = (total * (uint64_t)r + (uint64_t)world - 1) / (uint64_t)world;
    uint64_t i, b;
    t = 0;
    while( t + 1 < nthreads && before[t + 1] < target ) ++t;
    i = jobs[t].lo;
    b = before[t];
    while( i < n_total && b < target ) {
      b += (oo_pg_len(config, seed, i) + align - 1) / align * align;
      ++i;
    }
    firsts[r] = i < firsts[r - 1] ? firsts[r - 1] : i;
  }
  return 0;
}
