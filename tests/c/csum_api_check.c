/* SPDX-License-Identifier: BSD-2-Clause */
/*
 * csum_api_check.c -- a plain C caller of the boundary's host-pure
 * checksum verifiers (include/oo_gpu_rx.h), built with gcc
 * against that header and the system's wire-header structs only, linked
 * with -loo_gpu_rx.  It replays vectors whose verdicts the reference's own
 * checksum.c produced (tests/golden/ref_csum_vectors.npz, written to a flat
 * file by tests/test_csum_api.py) through every entry-point shape:
 * ef_{udp,tcp}_checksum[_ip6]_is_correct with 1-3 iovec pieces (odd splits
 * and empty pieces: ip_csum64_partialv's carry, checksum.c:134-159), the
 * _ipx forms, and ci_ip_csum_correct's IPv4 header check.
 *
 *   csum_api_check <l4-vectors> <ip-vectors>
 *
 * Prints "checked N mismatches M" and exits non-zero on any mismatch.
 */
#include <linux/ipv6.h>
#include <netinet/ip.h>
#include <netinet/tcp.h>
#include <netinet/udp.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/uio.h>

#include "oo_gpu_rx.h"

static int rd(FILE* f, void* p, size_t n) { return fread(p, 1, n, f) == n; }

static int l4_verdict(int af, int proto, const uint8_t* l3, const uint8_t* l4,
                      const uint8_t* pay, uint32_t paylen, int shape)
{
  struct iovec iov[3];
  int n = 1;
  /* shape 0: one piece; 1: two, split at an odd point; 2: three, the middle
   * one empty; 3: the _ipx form. */
  uint32_t a = paylen / 3 | 1u, b;
  if( a > paylen ) a = paylen;
  iov[0].iov_base = (void*)pay;
  iov[0].iov_len = paylen;
  if( shape == 1 ) {
    iov[0].iov_len = a;
    iov[1].iov_base = (void*)(pay + a);
    iov[1].iov_len = paylen - a;
    n = 2;
  } else if( shape == 2 ) {
    b = (paylen - a) / 2;
    iov[0].iov_len = a;
    iov[1].iov_base = (void*)(pay + a);
    iov[1].iov_len = 0;
    iov[2].iov_base = (void*)(pay + a);
    iov[2].iov_len = paylen - a;
    (void)b;
    n = 3;
  }
  if( shape == 3 ) {
    if( proto == 17 )
      return oo_rx_udp_csum_ok_ipx(af == 6 ? AF_INET6 : AF_INET, l3,
                                   (const struct udphdr*)l4, pay, paylen);
    return oo_rx_tcp_csum_ok_ipx(af == 6 ? AF_INET6 : AF_INET, l3,
                                 (const struct tcphdr*)l4, pay, paylen);
  }
  if( proto == 17 )
    return af == 6 ?
      oo_rx_udp_csum_ok_ip6((const struct ipv6hdr*)l3, (const struct udphdr*)l4, iov, n) :
      oo_rx_udp_csum_ok((const struct iphdr*)l3, (const struct udphdr*)l4, iov, n);
  return af == 6 ?
    oo_rx_tcp_csum_ok_ip6((const struct ipv6hdr*)l3, (const struct tcphdr*)l4, iov, n) :
    oo_rx_tcp_csum_ok((const struct iphdr*)l3, (const struct tcphdr*)l4, iov, n);
}

int main(int argc, char** argv)
{
  FILE* f;
  uint32_t count, k;
  long checked = 0, bad = 0;
  if( argc != 3 ) {
    fprintf(stderr, "usage: %s <l4-vectors> <ip-vectors>\n", argv[0]);
    return 2;
  }
  /* L4 vectors: u32 count; per vector u32 af, proto, l3len, l4len, paylen,
   * ok, then the l3, l4 and payload bytes. */
  if( (f = fopen(argv[1], "rb")) == NULL || ! rd(f, &count, 4) ) return 2;
  for( k = 0; k < count; ++k ) {
    uint32_t m[6];
    uint8_t l3[64], l4[64], *pay;
    int shape;
    if( ! rd(f, m, sizeof(m)) || m[2] > 64 || m[3] > 64 ) return 2;
    pay = malloc(m[4] + 1);
    if( ! rd(f, l3, m[2]) || ! rd(f, l4, m[3]) || ! rd(f, pay, m[4]) ) return 2;
    for( shape = 0; shape < 4; ++shape ) {
      int got = l4_verdict((int)m[0], (int)m[1], l3, l4, pay, m[4], shape) != 0;
      ++checked;
      if( got != (int)m[5] ) {
        if( bad < 5 )
          fprintf(stderr, "vector %u shape %d: got %d want %u\n", k, shape, got, m[5]);
        ++bad;
      }
    }
    free(pay);
  }
  fclose(f);
  /* IPv4 header vectors: u32 count; per vector 60 header bytes, i32
   * max_ip_len, u32 ok. */
  if( (f = fopen(argv[2], "rb")) == NULL || ! rd(f, &count, 4) ) return 2;
  for( k = 0; k < count; ++k ) {
    uint8_t h[60];
    int32_t mx;
    uint32_t ok;
    int got;
    if( ! rd(f, h, 60) || ! rd(f, &mx, 4) || ! rd(f, &ok, 4) ) return 2;
    got = oo_rx_ip_csum_ok((const struct iphdr*)h, mx) != 0;
    ++checked;
    if( got != (int)ok ) {
      if( bad < 5 ) fprintf(stderr, "ip vector %u: got %d want %u\n", k, got, ok);
      ++bad;
    }
  }
  fclose(f);
  printf("checked %ld mismatches %ld\n", checked, bad);
  return bad ? 1 : 0;
}
