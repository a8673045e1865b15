/* SPDX-License-Identifier: BSD-2-Clause */
/*
 * ref_harness.c -- TEST INFRASTRUCTURE ONLY.  Exposes the reference's own
 * checksum and hash code, compiled unmodified from /root/reference by
 * oracle/Makefile into oracle/_ref/libref_rx.so, so the tests can pin the
 * oracle restatement against it.  Built only where /root/reference exists;
 * nothing on the GPU box or in the product needs it.
 *
 * Linked with the reference's src/lib/ciul/checksum.c (ef_*_checksum*,
 * ef_*_is_correct) and src/lib/citools/ip_csum_partial.c
 * (ci_ip_csum_partial); the hashes are the static inlines of
 * src/include/onload/hash.h and ci_ip_hdr_csum_finish of
 * src/include/ci/tools/ipcsum_base.h.
 */
#include <ci/internal/transport_config_opt.h>
#include <ci/tools.h>
#include <onload/hash.h>
#include <etherfabric/checksum.h>
#include <ci/tools/ipcsum_base.h>

/* __onload_hash{1,2,3} (hash.h:84-93, 137-144, 165-173). */
unsigned ref_hash3(unsigned la, unsigned lp, unsigned ra, unsigned rp, unsigned proto)
{ return __onload_hash3(la, lp, ra, rp, proto); }
unsigned ref_hash1(unsigned mask, unsigned la, unsigned lp, unsigned ra, unsigned rp,
                   unsigned proto)
{ return __onload_hash1(mask, la, lp, ra, rp, proto); }
unsigned ref_hash2(unsigned la, unsigned lp, unsigned ra, unsigned rp, unsigned proto)
{ return __onload_hash2(la, lp, ra, rp, proto); }

/* onload_addr_xor (hash.h:31-42) on a 16-byte ci_addr_t. */
unsigned ref_addr_xor(const void* a16)
{
  ci_addr_t a;
  memcpy(&a, a16, sizeof(a));
  return onload_addr_xor(a);
}

/* onload_hash3 / hash1 / hash2 with ci_addr_t arguments (IPv6 table). */
unsigned ref_onload_hash3(const void* la16, unsigned lp, const void* ra16, unsigned rp,
                          unsigned proto)
{
  ci_addr_t la, ra;
  memcpy(&la, la16, sizeof(la));
  memcpy(&ra, ra16, sizeof(ra));
  return onload_hash3(la, lp, ra, rp, proto);
}

/* The body of ci_ip_csum_correct (netif_event.c:80-94, a static function
 * the harness cannot link) from the reference's own pieces:
 * ci_ip_csum_partial + ci_ip_hdr_csum_finish. */
int ref_ip_hdr_csum_ok(const void* ip, int max_ip_len)
{
  const unsigned char* p = ip;
  int ihl4 = (p[0] & 0xf) << 2;
  int ip_len = (p[2] << 8) | p[3];
  unsigned csum;
  if( max_ip_len < ihl4 )
    return 0;
  if( max_ip_len < ip_len )
    return 0;
  csum = ci_ip_csum_partial(0, ip, ihl4);
  csum = ci_ip_hdr_csum_finish(csum);
  return csum == 0;
}

/* The checksum.h inline wrappers (checksum.h:246-308) as callable symbols. */
int ref_udp_ok(int af, const void* ipx, const void* udp, const void* pay, size_t n)
{ return ef_udp_checksum_ipx_is_correct(af == 6 ? AF_INET6 : AF_INET, ipx, udp, pay, n); }
int ref_tcp_ok(int af, const void* ipx, const void* tcp, const void* pay, size_t n)
{ return ef_tcp_checksum_ipx_is_correct(af == 6 ? AF_INET6 : AF_INET, ipx, tcp, pay, n); }
