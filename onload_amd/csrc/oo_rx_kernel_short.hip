// SPDX-License-Identifier: BSD-2-Clause
// rx_kernel for short-frame batches: the same tile loop with a 2-slot body
// ring, so a block needs less LDS and a CU holds 12 waves instead of 10
// (more waves to overlap the per-tile header and table-lookup chain, which
// bounds short frames; long frames need the 4-slot ring's bytes in flight),
// and per-group job sequences for the body: IMIX tiles mix job sizes, whose
// lockstep slots idle a fifth of the ring.
// Chosen per launch by oo_gpu_rx.cpp launch().
#undef OO_RX_RING
#define OO_RX_RING 2
#undef OO_RX_GSEQ
#define OO_RX_GSEQ 1
#define OO_RX_SHORT 1
#include "oo_rx_kernel.hip"
