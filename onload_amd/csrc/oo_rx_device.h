// SPDX-License-Identifier: BSD-2-Clause
//
// oo_rx_device.h -- layouts shared by the gfx950 kernels (oo_rx_kernel.hip)
// and the host side of the C ABI (oo_gpu_rx.cpp).  Internal; not installed.
#ifndef OO_RX_DEVICE_H
#define OO_RX_DEVICE_H

#include <stdint.h>

#include "../../include/oo_gpu_rx.h"

namespace oo_rx {

// IPv4 filter table: ci_netif_filter_table_entry_fast {id_and_state, laddr}
// (ip_shared_types.h:533-540) and _ext {route_count, lport}
// (ip_shared_types.h:545-548) as uint2 arrays.  IPv6 table:
// ci_ip6_netif_filter_table_entry {id, route_count, laddr[16]}
// (ip_shared_types.h:579-583).
struct Ip6Entry {
  int32_t id;
  int32_t route_count;
  uint32_t laddr[4];
};
static_assert(sizeof(Ip6Entry) == 24, "ip6 entry layout");
static_assert(sizeof(oo_gpu_rx_sock) == 48, "socket record layout");
static_assert(sizeof(oo_gpu_rx_result) == 32, "result record layout");
static_assert(sizeof(oo_gpu_pkt_desc) == 16, "descriptor layout");

struct uint2_ {
  uint32_t x, y;
};

// Kernel arguments (passed by value).
struct KParams {
  const uint8_t* frames;
  uint64_t frames_bytes;
  const oo_gpu_pkt_desc* desc;
  oo_gpu_rx_result* out;
  uint32_t* counters;  // OO_RX_R_COUNT u32, may be null
  uint32_t n;
  uint32_t ip4_mask;
  uint32_t ip6_mask;
  uint32_t max_socks;
#ifdef __HIPCC__
  const uint2* ip4;
  const uint2* ip4_ext;
#else
  const uint2_* ip4;
  const uint2_* ip4_ext;
#endif
  const Ip6Entry* ip6;
  const oo_gpu_rx_sock* socks;
  uint8_t hwport[OO_GPU_RX_MAX_INTF];
};

}  // namespace oo_rx

#endif
