/* SPDX-License-Identifier: BSD-2-Clause */
/*
 * ref_l4_harness.c -- TEST INFRASTRUCTURE ONLY.  Runs the reference's own
 * receive path for one frame at a time -- handle_rx_csum_bad, handle_rx_pkt
 * and ci_parse_rx_vlan (src/lib/transport/ip/netif_event.c, #included below
 * to reach its statics), ci_udp_handle_rx (udp_rx.c) and ci_tcp_handle_rx
 * (tcp_rx.c), the filter tables (netif_table.c, netif_table_ip6.c) and the
 * checksum code (ciul/checksum.c, citools/ip_csum_partial.c), all compiled
 * unmodified by oracle/Makefile -- to generate the fixtures that pin the
 * oracle's and the kernel's gates, lookup stages and future rules
 * (tests/golden/make_l4_golden.py).  This is SURVEY.md Appendix A's recipe.
 *
 * Linked as the reference links its unit tests (src/tests/unit/mmake.mk:
 * 80-99: non-PIE, --unresolved-symbols=ignore-all, the object under test
 * plus harness definitions of the functions it calls out to, as its
 * lib/transport/ip/tcp_rx.c unit test defines ci_netif_filter_for_each_match
 * and ci_netif_pkt_pass_to_kernel).  Here the lookups are the REAL table
 * walks, observed through ld --wrap:
 *   __wrap_ci_netif_filter_for_each_match[_ip6]
 *       count mode (the full handlers): runs the real walk with a counting
 *       callback, records {matches, first socket} per lookup stage and the
 *       stage-1 hash, and plays the deliver callback's part for the stage
 *       that matched -- TCP: rxp->pkt = NULL, UDP: state->delivered = 1 --
 *       returning 1 as the real callbacks do (tcp_rx.c:4644-4657,
 *       udp_rx.c:141-228);
 *       pass-through mode (the futures): the real walk with the caller's own
 *       callback (ci_udp_rx_deliver_to_future, ci_tcp_rx_deliver_to_future).
 *   __wrap_ci_udp_handle_rx / __wrap_ci_tcp_handle_rx
 *       record the L4 entry (offset, ip_paylen), run the real pre-future
 *       (udp_internal.h:58-103 / tcp_rx.h:150-184) in pass-through mode for
 *       an IPv4 packet, then the real handler in count mode.
 *   ci_netif_pkt_pass_to_kernel: records "kernel", returns 1.
 * Hidden (CI_HF) symbols the link cannot leave unresolved get
 * __builtin_trap() bodies generated from the linker's own list
 * (oracle/Makefile): none is reached -- reaching one kills the harness.
 *
 * Script (stdin), one command per line; every command prints one line:
 *   I log4 log6 nsocks nintf hwport0 ...        init (as ref_table_harness)
 *   S id af proto lport rport raddr flags hwports vlan
 *   A af sock laddr lport raddr rport proto     ci_netif_filter_insert
 *   P intf hexframe                             one frame ->
 *     "r handled kernel entry l4off ip_paylen n1 f1 n2 f2 n3 f3 hash fut
 *        | eth ipcsum udp udpset tcp proto | name=delta ..."
 *     entry 0: no L4 handler ran, else 6 / 17; nK fK per lookup stage K the
 *     handler ran (-1 -1 if it did not); hash: stage-1 hash_out (TCP);
 *     fut: the pre-future's socket (-1 none, -2 not run).
 *     Then what tells handle_rx_csum_bad's drop branches apart (several
 *     share a counter or none, netif_event.c:1024-1127), observed on the
 *     run: eth 4 / 6 / 0 -- its IPv4 or IPv6 branch ran (the IS_IP6 flag it
 *     clears or sets, seen over two runs with the flag preset both ways), or
 *     neither; ipcsum 1 if ci_ip_csum_partial ran (ci_ip_csum_correct,
 *     :80-94); udp / tcp -1 if ci_udp_csum_correct (udp_rx.c:101-121) /
 *     ef_tcp_checksum[_ip6]_is_correct (checksum.c:326-351) did not run, else
 *     its verdict; udpset 1 if pkt->pf.udp.pay_len was written (:1105); proto
 *     the protocol byte at the L3 offset ci_parse_rx_vlan left (-1: neither
 *     branch).  Last, every stack counter the frame changed, by name, with
 *     its delta: ni->state->stats_snapshot's ip / tcp / udp / tcp_ext groups
 *     (ip_stats_ops.h:165-291) and ni->state->stats (stats_def.h,
 *     CITP_STATS_NETIF_INC), over handle_rx_csum_bad and everything it ran
 *     -- except the pre-future helpers this harness runs only to observe them
 *     (their counter changes are undone).
 */
#include "netif_event.c"                  /* -I src/lib/transport/ip */
#include "udp_internal.h"

#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

static ci_netif ni_;
static ci_netif* ni = &ni_;
static int nsocks_;

/* ---- the record of one frame */
static struct {
  int kernel, entry, l4off, ip_paylen, stage, fut, tso;
  int n[3], first[3];
  unsigned hash;
} R;
static int g_passthrough;

static void hexbytes(const char* s, unsigned char* out, int n)
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
    hexbytes(s, (unsigned char*) a.ip6, 16);
  }
  else {
    unsigned char b[4];
    ci_uint32 v;
    hexbytes(s, b, 4);
    memcpy(&v, b, 4);
    a = CI_ADDR_FROM_IP4(v);
  }
  return a;
}

static int sock_id(ci_sock_cmn* s)
{
  return (int) OO_SP_TO_INT(oo_statep_to_sockp(ni, (oo_p) ((char*) s - (char*) ni->state)));
}

/* ---- the TCP timestamp-option fast layout (OO_RX_F_TSO), observed on the
 * reference's own code: ci_tcp_rx_deliver_to_conn (tcp_rx.c:4534-4546) takes
 * the layout test before anything that needs an established connection.  The
 * real callback runs on the stage-1 match in a forked child (its socket and
 * the stack are this process's copies, thrown away), with the rx packet's
 * timestamps preset to sentinels: the fast layout writes them and sets
 * CI_TCPT_FLAG_TSO; any other layout calls ci_tcp_parse_options (wrapped
 * here: reported at once).  Whatever the callback does after the test -- it
 * runs on a socket the harness never connected, so it may trap or fault --
 * ends the child and is reported from its signal handler.  1 / 0: the layout
 * test's outcome; -1: the child ended before reaching it; -2: not probed. */
#define PROBE_TS1 0xa5c3e1f7u
#define PROBE_TS2 0x5a3c1e7fu
static int g_probe_fd = -1, g_probe_slow;
static ciip_tcp_rx_pkt* g_probe_rxp;

static int probe_state(void)
{
  if( g_probe_slow )
    return 0;
  if( g_probe_rxp->timestamp != PROBE_TS1 || g_probe_rxp->timestamp_echo != PROBE_TS2 )
    return (g_probe_rxp->flags & CI_TCPT_FLAG_TSO) ? 1 : 0;
  return -1;
}

static void probe_report(int v)
{
  char ch = (char) ('0' + v + 1);
  ssize_t rc = write(g_probe_fd, &ch, 1);
  (void) rc;
  _exit(0);
}

static void probe_sig(int sig)
{
  (void) sig;
  probe_report(probe_state());
}

extern int __real_ci_tcp_parse_options(ci_netif*, ciip_tcp_rx_pkt*, ci_tcp_options*);
int __wrap_ci_tcp_parse_options(ci_netif* n, ciip_tcp_rx_pkt* rxp, ci_tcp_options* o)
{
  if( g_probe_fd >= 0 ) {
    g_probe_slow = 1;
    probe_report(0);
  }
  return __real_ci_tcp_parse_options(n, rxp, o);
}

static int tso_probe(ci_sock_cmn* s, int (*cb)(ci_sock_cmn*, void*), void* arg)
{
  int fds[2], v = -1;
  char ch;
  pid_t pid;
  if( pipe(fds) != 0 )
    return -1;
  fflush(stdout);
  pid = fork();
  if( pid == 0 ) {
    static const int sigs[] = { SIGSEGV, SIGBUS, SIGILL, SIGTRAP, SIGFPE, SIGABRT, SIGALRM };
    unsigned k;
    close(fds[0]);
    g_probe_fd = fds[1];
    g_probe_rxp = arg;
    for( k = 0; k < sizeof(sigs) / sizeof(sigs[0]); ++k )
      signal(sigs[k], probe_sig);
    alarm(2);
    g_probe_rxp->timestamp = PROBE_TS1;
    g_probe_rxp->timestamp_echo = PROBE_TS2;
    g_probe_rxp->flags = 0;
    (void) cb(s, arg);
    probe_report(probe_state());
  }
  close(fds[1]);
  if( pid > 0 && read(fds[0], &ch, 1) == 1 )
    v = ch - '0' - 1;
  close(fds[0]);
  if( pid > 0 )
    waitpid(pid, NULL, 0);
  return v;
}

/* ---- observed lookups */
struct count { int n; int first; };

static int count_cb(ci_sock_cmn* s, void* arg)
{
  struct count* c = arg;
  if( c->n++ == 0 )
    c->first = sock_id(s);
  return 0;
}

static int stage_done(unsigned proto, struct count* c, void* arg,
                      int (*cb)(ci_sock_cmn*, void*))
{
  int k = R.stage;
  if( k == 0 && proto == IPPROTO_TCP && c->n > 0 && cb == ci_tcp_rx_deliver_to_conn )
    R.tso = tso_probe(ID_TO_SOCK(ni, c->first), cb, arg);
  ++R.stage;
  if( k < 3 ) {
    R.n[k] = c->n;
    R.first[k] = c->first;
  }
  if( c->n == 0 )
    return 0;
  /* what the deliver callback that accepted the packet leaves behind */
  if( proto == IPPROTO_TCP )
    ((ciip_tcp_rx_pkt*) arg)->pkt = NULL;
  else
    ((struct ci_udp_rx_deliver_state*) arg)->delivered = 1;
  return 1;
}

extern int __real_ci_netif_filter_for_each_match(ci_netif*, unsigned, unsigned, unsigned,
                                                 unsigned, unsigned, int, int,
                                                 int (*)(ci_sock_cmn*, void*), void*,
                                                 ci_uint32*);
int __wrap_ci_netif_filter_for_each_match(ci_netif* n, unsigned la, unsigned lp, unsigned ra,
                                          unsigned rp, unsigned proto, int intf, int vlan,
                                          int (*cb)(ci_sock_cmn*, void*), void* arg,
                                          ci_uint32* hash_out)
{
  struct count c = { 0, -1 };
  ci_uint32 h = 0;
  if( g_passthrough )
    return __real_ci_netif_filter_for_each_match(n, la, lp, ra, rp, proto, intf, vlan, cb, arg,
                                                 hash_out);
  __real_ci_netif_filter_for_each_match(n, la, lp, ra, rp, proto, intf, vlan, count_cb, &c,
                                        hash_out ? &h : NULL);
  if( hash_out ) {
    *hash_out = h;
    if( R.stage == 0 )
      R.hash = h;
  }
  return stage_done(proto, &c, arg, cb);
}

#if CI_CFG_IPV6
extern int __real_ci_netif_filter_for_each_match_ip6(ci_netif*, const ci_addr_t*, unsigned,
                                                     const ci_addr_t*, unsigned, unsigned, int,
                                                     int, int (*)(ci_sock_cmn*, void*), void*,
                                                     ci_uint32*);
int __wrap_ci_netif_filter_for_each_match_ip6(ci_netif* n, const ci_addr_t* la, unsigned lp,
                                              const ci_addr_t* ra, unsigned rp, unsigned proto,
                                              int intf, int vlan,
                                              int (*cb)(ci_sock_cmn*, void*), void* arg,
                                              ci_uint32* hash_out)
{
  struct count c = { 0, -1 };
  ci_uint32 h = 0;
  if( g_passthrough )
    return __real_ci_netif_filter_for_each_match_ip6(n, la, lp, ra, rp, proto, intf, vlan, cb,
                                                     arg, hash_out);
  __real_ci_netif_filter_for_each_match_ip6(n, la, lp, ra, rp, proto, intf, vlan, count_cb, &c,
                                            hash_out ? &h : NULL);
  if( hash_out ) {
    *hash_out = h;
    if( R.stage == 0 )
      R.hash = h;
  }
  return stage_done(proto, &c, arg, cb);
}
#endif

/* ---- observed checksum checks */
static int g_ipcsum, g_udpcsum, g_tcpcsum;

extern unsigned __real_ci_ip_csum_partial(unsigned, const volatile void*, int);
unsigned __wrap_ci_ip_csum_partial(unsigned sum, const volatile void* buf, int bytes)
{
  g_ipcsum = 1;
  return __real_ci_ip_csum_partial(sum, buf, bytes);
}

extern int __real_ci_udp_csum_correct(ci_ip_pkt_fmt*, ci_udp_hdr*);
int __wrap_ci_udp_csum_correct(ci_ip_pkt_fmt* pkt, ci_udp_hdr* udp)
{
  int rc = __real_ci_udp_csum_correct(pkt, udp);
  g_udpcsum = rc != 0;
  return rc;
}

extern int __real_ef_tcp_checksum_is_correct(const struct iphdr*, const struct tcphdr*,
                                             const struct iovec*, int);
int __wrap_ef_tcp_checksum_is_correct(const struct iphdr* ip, const struct tcphdr* tcp,
                                      const struct iovec* iov, int iovlen)
{
  int rc = __real_ef_tcp_checksum_is_correct(ip, tcp, iov, iovlen);
  g_tcpcsum = rc != 0;
  return rc;
}

extern int __real_ef_tcp_checksum_ip6_is_correct(const struct ipv6hdr*, const struct tcphdr*,
                                                 const struct iovec*, int);
int __wrap_ef_tcp_checksum_ip6_is_correct(const struct ipv6hdr* ip6, const struct tcphdr* tcp,
                                          const struct iovec* iov, int iovlen)
{
  int rc = __real_ef_tcp_checksum_ip6_is_correct(ip6, tcp, iov, iovlen);
  g_tcpcsum = rc != 0;
  return rc;
}

/* ---- stack counters around a frame */
static ci_ip_stats g_ip0;
static ci_netif_stats g_ni0;

static void stats_save(ci_ip_stats* ip, ci_netif_stats* nst)
{
  memcpy(ip, &ni->state->stats_snapshot, sizeof(*ip));
  memcpy(nst, &ni->state->stats, sizeof(*nst));
}

static void stats_restore(const ci_ip_stats* ip, const ci_netif_stats* nst)
{
  memcpy(&ni->state->stats_snapshot, ip, sizeof(*ip));
  memcpy(&ni->state->stats, nst, sizeof(*nst));
}

static void stats_print_delta(const ci_ip_stats* a, const ci_netif_stats* na)
{
  const ci_ip_stats* b = &ni->state->stats_snapshot;
  const ci_netif_stats* nb = &ni->state->stats;
#define OO_STAT(desc, type, name, kind)                                        \
  if( b->GRP.name != a->GRP.name )                                             \
    printf(" " GRPS ".%s=%lld", #name, (long long) (b->GRP.name - a->GRP.name));
#define GRP ip
#define GRPS "ip"
#include <ci/internal/ip_stats_count_def.h>
#undef GRP
#undef GRPS
#define GRP tcp
#define GRPS "tcp"
#include <ci/internal/tcp_stats_count_def.h>
#undef GRP
#undef GRPS
#define GRP udp
#define GRPS "udp"
#include <ci/internal/udp_stats_count_def.h>
#undef GRP
#undef GRPS
#define GRP tcp_ext
#define GRPS "tcp_ext"
#include <ci/internal/tcp_ext_stats_count_def.h>
#undef GRP
#undef GRPS
#undef OO_STAT
#define OO_STAT(desc, type, name, kind)                                        \
  if( nb->name != na->name )                                                   \
    printf(" ni.%s=%lld", #name, (long long) (nb->name - na->name));
#include <ci/internal/stats_def.h>
#undef OO_STAT
}

/* ---- observed L4 entries */
extern void __real_ci_udp_handle_rx(ci_netif*, ci_ip_pkt_fmt*, ci_udp_hdr*, int);
void __wrap_ci_udp_handle_rx(ci_netif* n, ci_ip_pkt_fmt* pkt, ci_udp_hdr* udp, int ip_paylen)
{
  R.entry = IPPROTO_UDP;
  R.l4off = (int) ((char*) udp - PKT_START(pkt));
  R.ip_paylen = ip_paylen;
  if( oo_pkt_af(pkt) == AF_INET ) {
    struct ci_udp_rx_future fut;
    static ci_ip_stats ip;
    static ci_netif_stats nst;
    stats_save(&ip, &nst);
    g_passthrough = 1;
    ci_udp_handle_rx_pre_future(n, pkt, udp, ip_paylen, CI_ETHERTYPE_IP, &fut);
    g_passthrough = 0;
    stats_restore(&ip, &nst);
    R.fut = fut.socket ? sock_id(&fut.socket->s) : -1;
  }
  __real_ci_udp_handle_rx(n, pkt, udp, ip_paylen);
}

extern void __real_ci_tcp_handle_rx(ci_netif*, struct ci_netif_poll_state*, ci_ip_pkt_fmt*,
                                    ci_tcp_hdr*, int);
void __wrap_ci_tcp_handle_rx(ci_netif* n, struct ci_netif_poll_state* ps, ci_ip_pkt_fmt* pkt,
                             ci_tcp_hdr* tcp, int ip_paylen)
{
  R.entry = IPPROTO_TCP;
  R.l4off = (int) ((char*) tcp - PKT_START(pkt));
  R.ip_paylen = ip_paylen;
  if( oo_pkt_af(pkt) == AF_INET ) {
    struct ci_tcp_rx_future fut;
    static ci_ip_stats ip;
    static ci_netif_stats nst;
    stats_save(&ip, &nst);
    g_passthrough = 1;
    ci_tcp_handle_rx_pre_future(n, pkt, tcp, ip_paylen, &fut);
    g_passthrough = 0;
    stats_restore(&ip, &nst);
    R.fut = fut.socket ? sock_id(fut.socket) : -1;
  }
  __real_ci_tcp_handle_rx(n, ps, pkt, tcp, ip_paylen);
}

/* The harness's own definition, as the reference's tcp_rx unit test has. */
int ci_netif_pkt_pass_to_kernel(ci_netif* n, ci_ip_pkt_fmt* pkt)
{
  (void) n;
  (void) pkt;
  R.kernel = 1;
  return 1;
}

/* ---- setup */
static void do_init(int log4, int log6, int nsocks, int nintf, int* hw)
{
  unsigned n4 = 1u << log4, n6 = 1u << log6, i;
  size_t state_bytes = (sizeof(ci_netif_state) + 4095) & ~(size_t) 4095;
  char* base = calloc(1, state_bytes + (size_t) nsocks * EP_BUF_SIZE);
  ci_netif_state* st = (ci_netif_state*) base;
  memset(ni, 0, sizeof(*ni));
  ni->state = st;
  nsocks_ = nsocks;
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
                    const char* raddr, unsigned flags, unsigned long long hwports, int vlan)
{
  ci_sock_cmn* s = ID_TO_SOCK(ni, id);
  memset(s, 0, EP_BUF_SIZE);
  if( af == 6 ) {
    s->pkt.ether_type = CI_ETHERTYPE_IP6;
    hexbytes(raddr, (unsigned char*) s->pkt.ipx.ip6.daddr, 16);
    s->pkt.ipx.ip6.next_hdr = (unsigned char) proto;
  }
  else {
    unsigned char b[4];
    s->pkt.ether_type = CI_ETHERTYPE_IP;
    hexbytes(raddr, b, 4);
    memcpy(&s->pkt.ipx.ip4.ip_daddr_be32, b, 4);
    s->pkt.ipx.ip4.ip_protocol = (unsigned char) proto;
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
  /* Every receive queue has room: ci_udp_rx_deliver_to_future's recvq
   * test (udp_internal.h:47-48) then depends on the tables alone. */
  if( proto == IPPROTO_UDP )
    SOCK_TO_UDP(s)->stats.max_recvq_pkts = 1u << 30;
  printf("ok\n");
}

/* ---- one frame through handle_rx_csum_bad */
static ci_ip_pkt_fmt* frame_pkt(int intf, const char* hex, int len, int ip6_preset)
{
  static ci_ip_pkt_fmt* pkt;
  if( pkt == NULL )
    pkt = aligned_alloc(4096, 64 * 1024);
  memset(pkt, 0, sizeof(*pkt));
  pkt->pkt_start_off = 0;
  pkt->pkt_eth_payload_off = PKT_START_OFF_BAD;
  pkt->frag_next = OO_PP_NULL;
  pkt->refcount = 1 << 20;
  pkt->intf_i = (ci_int16) intf;
  if( ip6_preset )
    pkt->flags |= CI_PKT_FLAG_IS_IP6;
  pkt->pf.udp.pay_len = 0xdeadbeefu;
  hexbytes(hex, (unsigned char*) PKT_START(pkt), len);
  return pkt;
}

static void do_frame(int intf, const char* hex)
{
  static struct ci_netif_poll_state ps;
  ci_ip_pkt_fmt* pkt;
  int len = (int) strlen(hex) / 2, handled, i, eth = 0, udpset, proto = -1, f1, f2;
  int ipcsum, udpc, tcpc;
  if( len > 64 * 1024 - (int) CI_MEMBER_OFFSET(ci_ip_pkt_fmt, dma_start) - 64 ) {
    printf("toolong\n");
    return;
  }
  /* Run 1 (IS_IP6 preset): the record, the counters, the checks. */
  pkt = frame_pkt(intf, hex, len, 1);
  memset(&R, 0, sizeof(R));
  for( i = 0; i < 3; ++i )
    R.n[i] = R.first[i] = -1;
  R.fut = -2;
  R.tso = -2;
  g_ipcsum = 0;
  g_udpcsum = g_tcpcsum = -1;
  stats_save(&g_ip0, &g_ni0);
  handled = handle_rx_csum_bad(ni, &ps, pkt, len);
  f1 = (pkt->flags & CI_PKT_FLAG_IS_IP6) != 0;
  udpset = pkt->pf.udp.pay_len != 0xdeadbeefu;
  ipcsum = g_ipcsum;
  udpc = g_udpcsum;
  tcpc = g_tcpcsum;
  printf("r %d %d %d %d %d %d %d %d %d %d %d %u %d %d", handled, R.kernel, R.entry, R.l4off,
         R.ip_paylen, R.n[0], R.first[0], R.n[1], R.first[1], R.n[2], R.first[2], R.hash,
         R.fut, R.tso);
  /* Run 2 (IS_IP6 clear), a dropped frame only (no handler runs): which
   * address-family branch wrote the flag.  Its counters are undone. */
  if( ! handled ) {
    static ci_ip_stats ip;
    static ci_netif_stats nst;
    stats_save(&ip, &nst);
    pkt = frame_pkt(intf, hex, len, 0);
    (void) handle_rx_csum_bad(ni, &ps, pkt, len);
    f2 = (pkt->flags & CI_PKT_FLAG_IS_IP6) != 0;
    stats_restore(&ip, &nst);
    eth = (f1 && f2) ? 6 : (! f1 && ! f2) ? 4 : 0;
    if( eth && pkt->pkt_eth_payload_off != PKT_START_OFF_BAD ) {
      const unsigned char* l3 = (const unsigned char*) PKT_START(pkt) + pkt->pkt_eth_payload_off;
      proto = l3[eth == 4 ? 9 : 6];
    }
  }
  printf(" | %d %d %d %d %d %d |", eth, ipcsum, udpc, udpset, tcpc, proto);
  stats_print_delta(&g_ip0, &g_ni0);
  printf("\n");
}

int main(void)
{
  static char line[1 << 16];
  char a[64], b[64];
  while( fgets(line, sizeof(line), stdin) ) {
    int af, id, proto, vlan, rc, intf;
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
                 &rport, a, &flags, &hw, &vlan) != 9 || id < 0 || id >= nsocks_ )
        return 2;
      do_sock(id, af, proto, lport, rport, a, flags, hw, vlan);
      break;
    case 'A': {
      ci_addr_t l, r;
      if( sscanf(line + 1, "%d %d %63s %u %63s %u %d", &af, &id, a, &lport, b, &rport,
                 &proto) != 7 )
        return 2;
      l = addr_of(af, a);
      r = addr_of(af, b);
      rc = ci_netif_filter_insert(ni, OO_SP_FROM_INT(ni, id),
                                  af == 6 ? AF_SPACE_FLAG_IP6 : AF_SPACE_FLAG_IP4,
                                  l, lport, r, rport, proto);
      printf("%d\n", rc);
      break;
    }
    case 'P': {
      char* hex = line + 1;
      char* end;
      intf = (int) strtol(hex, &end, 10);
      while( *end == ' ' )
        ++end;
      end[strcspn(end, "\r\n")] = 0;
      do_frame(intf, end);
      break;
    }
    default:
      break;
    }
    fflush(stdout);
  }
  return 0;
}
