// SPDX-License-Identifier: BSD-2-Clause
//
// oo_rx_csum.cpp -- the boundary's host-pure checksum verifiers (SURVEY.md
// §8(b)): the same argument shapes as the reference's public C API for this
// path, so a caller that verifies one packet on the CPU (a packet outside a
// batch, a retransmitted segment, a test) gets the GPU path's verdicts.
//
//   oo_rx_ip_csum_ok           ci_ip_csum_correct  src/lib/transport/ip/netif_event.c:80-94
//                              (ci_ip_csum_partial src/lib/citools/ip_csum_partial.c:20-39,
//                               ci_ip_hdr_csum_finish src/include/ci/tools/ipcsum_base.h:10-14)
//   oo_rx_udp_csum_ok[_ip6]    ef_udp_checksum[_ip6]_is_correct  src/lib/ciul/checksum.c:298-324
//   oo_rx_tcp_csum_ok[_ip6]    ef_tcp_checksum[_ip6]_is_correct  checksum.c:326-351
//   oo_rx_{udp,tcp}_csum_ok_ipx   ef_{udp,tcp}_checksum_ipx_is_correct
//                              src/include/etherfabric/checksum.h:246-308
//
// Arithmetic.  The reference folds 64-bit add-with-carry partial sums of the
// little-endian 16-bit words (checksum.c:53-174); each of its steps keeps
// the sum's residue mod 0xffff and none turns a non-zero sum into zero, and
// the pseudo-header makes the sum non-zero, so "the folded complement is 0"
// is exactly "the word sum is 0 mod 0xffff" -- the verdict the gfx950
// kernel computes too.  The iovec walk pairs bytes across element
// boundaries as ip_csum64_partialv does (:134-159): an element that ends on
// an odd byte leaves it as a word's low byte and the next element's first
// byte is that word's high byte.
//
// No allocation, no state, no GPU: thread-safe, callable on any host.
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#include <sys/uio.h>

#include "../../include/oo_gpu_rx.h"

namespace {

constexpr int AF_INET6_ = 10;  // AF_INET6 (Linux)

// Sum of the little-endian 16-bit words of a byte stream fed in pieces.
struct WordSum {
  uint64_t s = 0;
  bool odd = false;  // the last piece ended half-way into a word
  void add(const uint8_t* p, size_t n) {
    if (n == 0) return;
    if (odd) {
      s += (uint64_t)p[0] << 8;
      ++p;
      --n;
    }
    size_t k = 0;
    for (; k + 8 <= n; k += 8) {
      uint64_t w;
      memcpy(&w, p + k, 8);
      s += (w & 0xffffu) + ((w >> 16) & 0xffffu) + ((w >> 32) & 0xffffu) + (w >> 48);
    }
    for (; k + 2 <= n; k += 2) s += (uint64_t)p[k] | ((uint64_t)p[k + 1] << 8);
    odd = k < n;
    if (odd) s += p[k];
  }
};

inline uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
inline uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }

bool residue_zero(uint64_t s) { return s % 0xffffu == 0; }

// The pseudo-header word sums (checksum.c:215-223, 304-305, 334-335).
uint64_t pseudo4(const uint8_t* ip, uint16_t len_be_as_le, uint32_t proto) {
  WordSum w;
  w.add(ip + 12, 8);  // saddr, daddr
  return w.s + len_be_as_le + (proto << 8);
}
uint64_t pseudo6(const uint8_t* ip6, uint16_t len_le, uint32_t proto) {
  WordSum w;
  w.add(ip6 + 8, 32);  // saddr, daddr
  return w.s + len_le + (proto << 8);
}

int l4_ok(uint64_t pseudo, const uint8_t* l4, size_t l4_hlen, const struct iovec* iov,
          int iovlen) {
  WordSum w;
  w.s = pseudo;
  w.add(l4, l4_hlen);
  for (int i = 0; i < iovlen; ++i)
    w.add(static_cast<const uint8_t*>(iov[i].iov_base), iov[i].iov_len);
  return residue_zero(w.s) ? 1 : 0;
}

}  // namespace

extern "C" {

int oo_rx_ip_csum_ok(const struct iphdr* ip, int max_ip_len) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(ip);
  const int ihl4 = (p[0] & 0xf) * 4;
  if (max_ip_len < ihl4) return 0;
  if (max_ip_len < (int)be16(p + 2)) return 0;
  uint32_t s = 0;  // a 32-bit accumulator, as ci_ip_csum_partial
  for (int k = 0; k + 1 < ihl4; k += 2) s += rd16(p + k);
  // ci_ip_hdr_csum_finish: ~fold(s) == 0 <=> s != 0 && s == 0 mod 0xffff
  return (s != 0 && s % 0xffffu == 0) ? 1 : 0;
}

int oo_rx_udp_csum_ok(const struct iphdr* ip, const struct udphdr* udp,
                      const struct iovec* iov, int iovlen) {
  const uint8_t* u = reinterpret_cast<const uint8_t*>(udp);
  return l4_ok(pseudo4(reinterpret_cast<const uint8_t*>(ip), rd16(u + 4), 17), u, 8, iov, iovlen);
}

int oo_rx_udp_csum_ok_ip6(const struct ipv6hdr* ip6, const struct udphdr* udp,
                          const struct iovec* iov, int iovlen) {
  const uint8_t* u = reinterpret_cast<const uint8_t*>(udp);
  return l4_ok(pseudo6(reinterpret_cast<const uint8_t*>(ip6), rd16(u + 4), 17), u, 8, iov,
               iovlen);
}

int oo_rx_tcp_csum_ok(const struct iphdr* ip, const struct tcphdr* tcp,
                      const struct iovec* iov, int iovlen) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(ip);
  const uint8_t* t = reinterpret_cast<const uint8_t*>(tcp);
  // htonl((IPPROTO_TCP << 16) | paylen), paylen a u16 (checksum.c:330-334)
  const uint16_t paylen = (uint16_t)(be16(p + 2) - (p[0] & 0xf) * 4);
  const uint16_t paylen_le = (uint16_t)((paylen >> 8) | (paylen << 8));
  return l4_ok(pseudo4(p, paylen_le, 6), t, (size_t)(t[12] >> 4) * 4, iov, iovlen);
}

int oo_rx_tcp_csum_ok_ip6(const struct ipv6hdr* ip6, const struct tcphdr* tcp,
                          const struct iovec* iov, int iovlen) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(ip6);
  const uint8_t* t = reinterpret_cast<const uint8_t*>(tcp);
  return l4_ok(pseudo6(p, rd16(p + 4), 6), t, (size_t)(t[12] >> 4) * 4, iov, iovlen);
}

int oo_rx_udp_csum_ok_ipx(int af, const void* ipx, const struct udphdr* udp,
                          const void* payload, size_t payload_len) {
  struct iovec iov;
  iov.iov_base = const_cast<void*>(payload);
  iov.iov_len = payload_len;
  return af == AF_INET6_
             ? oo_rx_udp_csum_ok_ip6(static_cast<const struct ipv6hdr*>(ipx), udp, &iov, 1)
             : oo_rx_udp_csum_ok(static_cast<const struct iphdr*>(ipx), udp, &iov, 1);
}

int oo_rx_tcp_csum_ok_ipx(int af, const void* ipx, const struct tcphdr* tcp,
                          const void* payload, size_t payload_len) {
  struct iovec iov;
  iov.iov_base = const_cast<void*>(payload);
  iov.iov_len = payload_len;
  return af == AF_INET6_
             ? oo_rx_tcp_csum_ok_ip6(static_cast<const struct ipv6hdr*>(ipx), tcp, &iov, 1)
             : oo_rx_tcp_csum_ok(static_cast<const struct iphdr*>(ipx), tcp, &iov, 1);
}

}  // extern "C"
