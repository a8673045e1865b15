/* SPDX-License-Identifier: BSD-2-Clause */
/*
 * poll_bench.c -- the deployed call shape of the batched RX branch
 * (include/oo_rx_poll.h): oo_rx_poll_evs over the RX events of an AF_XDP-
 * shaped pool (one frame per 2048-B buffer at headroom 192, host memory),
 * evs_per_poll events per call, timed per call, with the GPU context and the
 * shim as a C integration would use them (no-op callbacks that count).
 * Beside it, the per-event CPU loop it replaces: the oracle's restatement of
 * handle_rx_csum_bad -> handle_rx_pkt -> ci_{udp,tcp}_handle_rx
 * (oracle/rx_oracle.c, one frame at a time on one core, as
 * ci_netif_poll_evq's loop runs, netif_event.c:1709-1742).  The oracle is
 * linked only as that baseline.
 *
 *   tools/poll_bench <config> <frames> <evs_per_poll> [...]
 *
 * One JSON line per (evs_per_poll, mode); mode: gather (frames copied into
 * the shim's registered buffer), zero_copy (the pool registered, frames
 * read in place), or zero_copy_crossover (zero copy with
 * OO_RX_POLL_CROSSOVER: a chunk the cost model prices below the device
 * batch goes back through other_ev, and this program's other_ev runs the
 * per-event CPU loop on it inside the timed poll -- the deployed shape).
 * The crossover model's defaults (src/shim/oo_rx_poll.c gpu_pays) are fitted
 * to these lines.
 */
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/mman.h>
#include <string.h>
#include <time.h>

#include "oo_gpu_rx.h"
#include "oo_rx_poll.h"
#include "../onload_amd/csrc/oo_pktgen.h"
#include "../oracle/rx_oracle.h"

#define BUF 2048
#define HEADROOM 192

static double now_us(void)
{
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static int cmp_d(const void* a, const void* b)
{
  double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : x > y;
}

struct tally {
  uint64_t calls, cpu_events;
  oo_or_tables* ot;       /* the per-event loop's tables (other_ev)        */
  const uint8_t* pool;
};
static int cb_future(void* a, uint32_t id, const uint8_t* f, const oo_gpu_rx_result* r,
                     const oo_rx_poll_future* fu)
{ (void)id; (void)f; (void)r; (void)fu; ++((struct tally*)a)->calls; return 0; }
static void cb_h(void* a, uint32_t id, const uint8_t* f, const oo_gpu_rx_result* r)
{ (void)id; (void)f; (void)r; ++((struct tally*)a)->calls; }
/* An event handed back: the caller's loop transforms it, one at a time. */
static void cb_other(void* a, const oo_rx_poll_ev* e)
{
  struct tally* t = a;
  oo_gpu_rx_result r;
  ++t->calls;
  ++t->cpu_events;
  oo_or_rx_one(t->ot, t->pool + (uint64_t)e->rq_id * BUF + e->ofs, e->len, e->intf_i, &r);
}

int main(int argc, char** argv)
{
  int cfg, n, i, k, nf, ns, rc;
  oo_pg_filter* filters;
  oo_gpu_rx_sock* socks;
  uint8_t *packed, *pool;
  oo_gpu_pkt_desc* desc;
  oo_rx_poll_ev* evs;
  oo_gpu_rx_ctx* gpu;
  oo_gpu_rx_cfg gc;
  oo_or_tables* ot;
  uint64_t seed, need, pool_bytes;
  uint8_t hw0 = 0;
  double cpu_ns, mean_len = 0;
  if( argc < 4 ) {
    fprintf(stderr, "usage: %s config frames evs_per_poll...\n", argv[0]);
    return 2;
  }
  /* the process setting INTEGRATION.md §6 recommends for the context's owner
   * (kernel arguments read from HBM, not over PCIe), before the runtime
   * starts; an explicit value in the environment wins */
  setenv("HIP_FORCE_DEV_KERNARG", "1", 0);
  cfg = atoi(argv[1]);
  n = atoi(argv[2]);
  filters = calloc(8192, sizeof(*filters));
  socks = calloc(8192, sizeof(*socks));
  nf = oo_pg_world(cfg, filters, 8192, socks, 8192, &ns);
  if( nf < 0 )
    return 2;
  seed = oo_pg_default_seed(cfg);
  need = oo_pg_bytes(cfg, seed, 0, (uint32_t)n, 64);
  packed = malloc(need);
  desc = malloc(sizeof(*desc) * n);
  if( oo_pg_gen(cfg, seed, 0, (uint32_t)n, 64, packed, need, desc, 8) != need )
    return 3;
  /* The AF_XDP layout: frame i in buffer i at HEADROOM (single-buffer frames
   * only: the shim hands a frame that overruns its buffer back). */
  /* (whole pages of its own, as oo_gpu_rx_host_register requires) */
  pool_bytes = ((uint64_t)n * BUF + 4095) & ~(uint64_t)4095;
  pool = mmap(NULL, pool_bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if( pool == MAP_FAILED )
    return 3;
  evs = calloc(n, sizeof(*evs));
  for( i = 0; i < n; ++i ) {
    uint32_t len = desc[i].len;
    if( len > BUF - HEADROOM )
      len = BUF - HEADROOM;
    memcpy(pool + (uint64_t)i * BUF + HEADROOM, packed + desc[i].frame_off, len);
    evs[i].rq_id = (uint32_t)i;
    evs[i].ofs = HEADROOM;
    evs[i].len = (uint16_t)len;
    evs[i].flags = OO_RX_EV_SOP;
    evs[i].intf_i = 0;
    mean_len += len;
  }
  mean_len /= n;

  /* The per-event CPU loop: one frame at a time, one core. */
  ot = oo_or_tables_new(16, 14, 8192, &hw0, 1);
  for( i = 0; i < ns; ++i )
    oo_or_sock_set(ot, i, &socks[i]);
  for( i = 0; i < nf; ++i )
    oo_or_insert(ot, filters[i].af, filters[i].laddr, filters[i].lport_be,
                 filters[i].raddr_any ? NULL : filters[i].raddr, filters[i].rport_be,
                 filters[i].proto, filters[i].sock);
  {
    oo_gpu_rx_result r;
    double t0 = now_us();
    for( i = 0; i < n; ++i )
      oo_or_rx_one(ot, pool + (uint64_t)i * BUF + HEADROOM, evs[i].len, 0, &r);
    cpu_ns = (now_us() - t0) * 1e3 / n;
  }

  memset(&gc, 0, sizeof(gc));
  gc.device = 0;
  gc.max_socks = 8192;
  gc.ip4_table_log2 = 16;
  gc.ip6_table_log2 = 14;
  gc.n_intf = 1;
  gc.host_stage_bytes = (uint64_t)BUF * 65536;
  gc.host_stage_pkts = 65536;
  if( (rc = oo_gpu_rx_open(&gpu, &gc)) != 0 ) {
    fprintf(stderr, "oo_gpu_rx_open: %d\n", rc);
    return 4;
  }
  for( i = 0; i < ns; ++i )
    oo_gpu_rx_sock_set(gpu, i, &socks[i]);
  for( i = 0; i < nf; ++i )
    oo_gpu_rx_table_insert(gpu, filters[i].af, filters[i].laddr, filters[i].lport_be,
                           filters[i].raddr_any ? NULL : filters[i].raddr, filters[i].rport_be,
                           filters[i].proto, filters[i].sock);
  oo_gpu_rx_sync_tables(gpu, NULL);

  for( k = 3; k < argc; ++k ) {
    uint32_t epp = (uint32_t)atoi(argv[k]);
    int zc;
    for( zc = 0; zc < 3; ++zc ) {
      struct tally t = { 0, 0, ot, pool };
      oo_rx_poll_ops ops = { cb_future, cb_h, cb_h, cb_h, cb_other, &t };
      oo_rx_poll_cfg pc;
      oo_rx_poll_stats st;
      oo_rx_poll* p;
      uint32_t npoll = (uint32_t)((n + epp - 1) / epp), q;
      double* lat = malloc(sizeof(double) * npoll);
      double t0, total;
      memset(&pc, 0, sizeof(pc));
      pc.pkt_bufs = pool;
      pc.pkt_bufs_bytes = pool_bytes;
      pc.buf_size = BUF;
      pc.evs_per_poll = epp;
      pc.sw_verify = 1;
      pc.flags = zc ? OO_RX_POLL_ZERO_COPY : 0;
      if( zc == 2 )
        pc.flags |= OO_RX_POLL_CROSSOVER;
      if( (rc = oo_rx_poll_open(&p, gpu, &pc, &ops)) != 0 ) {
        fprintf(stderr, "oo_rx_poll_open: %d\n", rc);
        return 5;
      }
      memset(&st, 0, sizeof(st));
      /* warm: one pass */
      for( q = 0; q < npoll; ++q ) {
        uint32_t m = (uint32_t)n - q * epp < epp ? (uint32_t)n - q * epp : epp;
        if( oo_rx_poll_evs(p, evs + (uint64_t)q * epp, m, &st) != (int)m )
          return 6;
      }
      t0 = now_us();
      for( q = 0; q < npoll; ++q ) {
        uint32_t m = (uint32_t)n - q * epp < epp ? (uint32_t)n - q * epp : epp;
        double a = now_us();
        oo_rx_poll_evs(p, evs + (uint64_t)q * epp, m, &st);
        lat[q] = now_us() - a;
      }
      total = now_us() - t0;
      qsort(lat, npoll, sizeof(double), cmp_d);
      printf("{\"config\": %d, \"frames\": %d, \"evs_per_poll\": %u, \"mode\": \"%s\", "
             "\"zero_copy_active\": %d, \"polls\": %u, \"poll_us_median\": %.2f, "
             "\"poll_us_p99\": %.2f, \"mpps\": %.3f, \"cpu_per_event_ns\": %.1f, "
             "\"cpu_mpps_1core\": %.3f, \"cpu_poll_us_equiv\": %.2f, \"callbacks\": %llu, "
             "\"handed_back\": %llu, \"mean_len\": %.1f}\n",
             cfg, n, epp, zc == 2 ? "zero_copy_crossover" : zc ? "zero_copy" : "gather",
             oo_rx_poll_zero_copy(p), npoll,
             lat[npoll / 2], lat[(npoll * 99) / 100 < npoll ? (npoll * 99) / 100 : npoll - 1],
             n / total, cpu_ns, 1e3 / cpu_ns, cpu_ns * epp * 1e-3,
             (unsigned long long)t.calls, (unsigned long long)st.n_handback / 2, mean_len);
      fflush(stdout);
      oo_rx_poll_close(p);
      free(lat);
    }
  }
  oo_gpu_rx_close(gpu);
  munmap(pool, pool_bytes);
  oo_or_tables_free(ot);
  return 0;
}
