/* SPDX-License-Identifier: BSD-2-Clause */
/*
 * ref_table_harness.c -- TEST INFRASTRUCTURE ONLY.  Drives the reference's
 * own filter-table code -- src/lib/transport/ip/netif_table.c and
 * netif_table_ip6.c, compiled unmodified by oracle/Makefile -- with a script
 * of table operations, to generate the fixtures that pin the table half of
 * the oracle and of the product (tests/golden/make_table_golden.py).
 *
 * Built and linked as the reference builds and links its unit tests
 * (src/tests/unit/mmake.mk:80-99): a debug build (ci_assert live, so the
 * table code checks its own invariants on every operation), a non-PIE
 * executable with --unresolved-symbols=ignore-all, and the reference's own
 * src/tests/unit/stubs.c for the log mask, ci_log and __ci_fail.  The
 * unresolved dump helpers (ip_addr_str, sock_raddr) are on paths the
 * harness never takes.
 *
 * The ci_netif it builds holds exactly what the table code reads: the
 * state block with ep_ofs / n_ep_bufs / intf_i_to_hwport / stats, 1024-B
 * socket buffers at ep_ofs + id * EP_BUF_SIZE (ip_shared_ops.h:270-332)
 * whose ipcache carries the socket's raddr / ports / protocol
 * (ip.h:1309-1340), and the three tables initialised as
 * ci_netif_filter_init (netif_table.c:592-611) and the IPv6 initialiser
 * (netif_table_ip6.c, EMPTY = -2) would.
 *
 * Script (stdin, one command per line; addresses as hex, "-" = none):
 *   I log4 log6 nsocks nintf hwport0 ...        init
 *   S id af proto lport rport raddr flags hwports vlan
 *                                               socket fields
 *                                               (flags: 1 CONNECTED, 2 bind2dev)
 *   A af sock laddr lport raddr rport proto     ci_netif_filter_insert -> rc
 *   R af sock laddr lport raddr rport proto     ci_netif_filter_remove
 *   L af laddr lport raddr rport proto          __ci_ip4_netif_filter_lookup /
 *                                               ci_ip6_netif_filter_lookup -> rc
 *   M af laddr lport raddr rport proto intf vlan
 *                                               ci_netif_filter_for_each_match{,_ip6}
 *                                               with a counting callback ->
 *                                               n first hash
 *   D                                           every slot that differs from
 *                                               its initial value
 * Ports are network-order values in host integers; every output is one line.
 */
#include <ci/internal/transport_config_opt.h>
#include <ci/internal/ip.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* not in the public headers: netif_table.c:617 */
extern int __ci_ip4_netif_filter_lookup(ci_netif* netif, unsigned laddr, unsigned lport,
                                        unsigned raddr, unsigned rport, unsigned protocol);

static ci_netif ni_;
static ci_netif* ni = &ni_;

static void hexaddr(const char* s, unsigned char* out, int n)
{
  int i;
  memset(out, 0, n);
  if( s[0] == '-' )
    return;
  for( i = 0; i < n && s[2 * i] && s[2 * i + 1]; ++i ) {
    unsigned v;
    sscanf(s + 2 * i, "%2x", &v);
    out[i] = (unsigned char) v;
  }
}

static ci_addr_t addr_of(int af, const char* s)
{
  ci_addr_t a;
  memset(&a, 0, sizeof(a));
  if( af == 6 ) {
    hexaddr(s, (unsigned char*) a.ip6, 16);
  }
  else {
    unsigned char b[4];
    ci_uint32 v;
    hexaddr(s, b, 4);
    memcpy(&v, b, 4);
    a = CI_ADDR_FROM_IP4(v);
  }
  return a;
}

static void do_init(int log4, int log6, int nsocks, int nintf, int* hw)
{
  unsigned n4 = 1u << log4, n6 = 1u << log6, i;
  size_t state_bytes = (sizeof(ci_netif_state) + 4095) & ~(size_t) 4095;
  char* base = calloc(1, state_bytes + (size_t) nsocks * EP_BUF_SIZE);
  ci_netif_state* st = (ci_netif_state*) base;
  memset(ni, 0, sizeof(*ni));
  ni->state = st;
  st->lock.lock = CI_EPLOCK_LOCKED;  /* called under the stack lock */
  *(ci_uint32*) &st->ep_ofs = (ci_uint32) state_bytes;
  *(ci_uint32*) &st->n_ep_bufs = (ci_uint32) nsocks;
  for( i = 0; i < (unsigned) nintf && i < CI_CFG_MAX_INTERFACES; ++i )
    st->intf_i_to_hwport[i] = (ci_int8) hw[i];
  ni->filter_table = calloc(1, sizeof(ci_netif_filter_table) +
                               n4 * sizeof(ci_netif_filter_table_entry_fast));
  ni->filter_table_ext = calloc(n4, sizeof(ci_netif_filter_table_entry_ext));
  *(unsigned*) &ni->filter_table->table_size_mask = n4 - 1;
  for( i = 0; i < n4; ++i )
    ni->filter_table->table[i].__id_and_state = 2u << 30;  /* EMPTY, id 0 */
  ni->ip6_filter_table = calloc(1, sizeof(ci_ip6_netif_filter_table) +
                                   n6 * sizeof(ci_ip6_netif_filter_table_entry));
  *(unsigned*) &ni->ip6_filter_table->table_size_mask = n6 - 1;
  for( i = 0; i < n6; ++i )
    ni->ip6_filter_table->table[i].id = -2;               /* EMPTY */
  printf("ok\n");
}

static void do_sock(int id, int af, int proto, unsigned lport, unsigned rport,
                    const char* raddr, unsigned flags, unsigned long long hwports,
                    int vlan)
{
  ci_sock_cmn* s = ID_TO_SOCK(ni, id);
  memset(s, 0, EP_BUF_SIZE);
  if( af == 6 ) {
    s->pkt.ether_type = CI_ETHERTYPE_IP6;
    hexaddr(raddr, (unsigned char*) s->pkt.ipx.ip6.daddr, 16);
    s->pkt.ipx.ip6.next_hdr = (ci_uint8) proto;
  }
  else {
    unsigned char b[4];
    s->pkt.ether_type = CI_ETHERTYPE_IP;
    hexaddr(raddr, b, 4);
    memcpy(&s->pkt.ipx.ip4.ip_daddr_be32, b, 4);
    s->pkt.ipx.ip4.ip_protocol = (ci_uint8) proto;
  }
  ipcache_lport_be16(&s->pkt) = (ci_uint16) lport;
  ipcache_rport_be16(&s->pkt) = (ci_uint16) rport;
  if( flags & 1 )
    s->s_flags |= CI_SOCK_FLAG_CONNECTED;
  if( flags & 2 ) {
    s->rx_bind2dev_ifindex = 1;
    s->rx_bind2dev_hwports = hwports;
    s->rx_bind2dev_vlan = (ci_int16) vlan;
  }
  else {
    s->rx_bind2dev_ifindex = CI_IFID_BAD;
  }
  printf("ok\n");
}

struct count { int n; int first; };

static int count_cb(ci_sock_cmn* s, void* arg)
{
  struct count* c = arg;
  if( c->n++ == 0 )
    c->first = (int) OO_SP_TO_INT(oo_statep_to_sockp(ni, (oo_p) ((char*) s - (char*) ni->state)));
  return 0;
}

static void do_match(int af, const char* la, unsigned lport, const char* ra,
                     unsigned rport, int proto, int intf, int vlan)
{
  struct count c = { 0, -1 };
  ci_uint32 hash = 0;
  ci_addr_t l = addr_of(af, la), r = addr_of(af, ra);
  if( af == 6 )
    ci_netif_filter_for_each_match_ip6(ni, &l, lport, ra[0] == '-' ? NULL : &r, rport,
                                       proto, intf, vlan, count_cb, &c, &hash);
  else
    ci_netif_filter_for_each_match(ni, l.ip4, lport, r.ip4, rport, proto, intf, vlan,
                                   count_cb, &c, &hash);
  printf("%d %d %u\n", c.n, c.first, hash);
}

static void do_dump(void)
{
  unsigned i, n4 = ni->filter_table->table_size_mask + 1;
  unsigned n6 = ni->ip6_filter_table->table_size_mask + 1;
  for( i = 0; i < n4; ++i ) {
    ci_netif_filter_table_entry_fast* e = &ni->filter_table->table[i];
    ci_netif_filter_table_entry_ext* x = &ni->filter_table_ext[i];
    if( e->__id_and_state != (2u << 30) || e->laddr || x->route_count || x->lport )
      printf("d4 %u %u %u %d %u\n", i, e->__id_and_state, e->laddr,
             x->route_count, x->lport);
  }
  for( i = 0; i < n6; ++i ) {
    ci_ip6_netif_filter_table_entry* e = &ni->ip6_filter_table->table[i];
    int k, z = 1;
    for( k = 0; k < 16; ++k )
      z &= ((unsigned char*) e->laddr)[k] == 0;
    if( e->id != -2 || e->route_count || !z ) {
      printf("d6 %u %d %d ", i, e->id, e->route_count);
      for( k = 0; k < 16; ++k )
        printf("%02x", ((unsigned char*) e->laddr)[k]);
      printf("\n");
    }
  }
  printf("end\n");
}

int main(void)
{
  char line[512], a[64], b[64];
  while( fgets(line, sizeof(line), stdin) ) {
    int af, id, proto, intf, vlan, rc;
    unsigned lport, rport, flags;
    unsigned long long hw;
    switch( line[0] ) {
    case 'I': {
      int log4, log6, ns, nintf, hwp[CI_CFG_MAX_INTERFACES] = {0}, k, pos = 0, used;
      if( sscanf(line + 1, "%d %d %d %d%n", &log4, &log6, &ns, &nintf, &pos) < 4 )
        return 2;
      for( k = 0; k < nintf && k < CI_CFG_MAX_INTERFACES; ++k ) {
        if( sscanf(line + 1 + pos, "%d%n", &hwp[k], &used) < 1 )
          return 2;
        pos += used;
      }
      do_init(log4, log6, ns, nintf, hwp);
      break;
    }
    case 'S':
      if( sscanf(line + 1, "%d %d %d %u %u %63s %u %llu %d", &id, &af, &proto, &lport,
                 &rport, a, &flags, &hw, &vlan) != 9 )
        return 2;
      do_sock(id, af, proto, lport, rport, a, flags, hw, vlan);
      break;
    case 'A':
    case 'R': {
      ci_addr_t l, r;
      if( sscanf(line + 1, "%d %d %63s %u %63s %u %d", &af, &id, a, &lport, b, &rport,
                 &proto) != 7 )
        return 2;
      l = addr_of(af, a);
      r = addr_of(af, b);
      if( line[0] == 'A' ) {
        rc = ci_netif_filter_insert(ni, OO_SP_FROM_INT(ni, id),
                                    af == 6 ? AF_SPACE_FLAG_IP6 : AF_SPACE_FLAG_IP4,
                                    l, lport, r, rport, proto);
        printf("%d\n", rc);
      }
      else {
        ci_netif_filter_remove(ni, OO_SP_FROM_INT(ni, id),
                               af == 6 ? AF_SPACE_FLAG_IP6 : AF_SPACE_FLAG_IP4,
                               l, lport, r, rport, proto);
        printf("0\n");
      }
      break;
    }
    case 'L': {
      ci_addr_t l, r;
      if( sscanf(line + 1, "%d %63s %u %63s %u %d", &af, a, &lport, b, &rport, &proto) != 6 )
        return 2;
      l = addr_of(af, a);
      r = addr_of(af, b);
      if( af == 6 )
        rc = ci_ip6_netif_filter_lookup(ni, l, lport, r, rport, proto);
      else
        rc = __ci_ip4_netif_filter_lookup(ni, l.ip4, lport, r.ip4, rport, proto);
      printf("%d\n", rc);
      break;
    }
    case 'M':
      if( sscanf(line + 1, "%d %63s %u %63s %u %d %d %d", &af, a, &lport, b, &rport, &proto,
                 &intf, &vlan) != 8 )
        return 2;
      do_match(af, a, lport, b, rport, proto, intf, vlan);
      break;
    case 'D':
      do_dump();
      break;
    default:
      break;
    }
    fflush(stdout);
  }
  return 0;
}
