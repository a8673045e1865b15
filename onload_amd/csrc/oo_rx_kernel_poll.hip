// SPDX-License-Identifier: BSD-2-Clause
// rx_kernel for a poll's batch (at most oo_gpu_rx.cpp SMALL_N packets): the
// same tile loop with a 12-slot body ring, so a tile's frames up to 1.5 KiB
// are requested whole with their header windows (one PCIe round trip for a
// batch read in place, where the 4-slot ring chains three), and a completion
// word written by the kernel itself (oo_rx_kernel.hip "The poll instance";
// DESIGN.md §5e).
#undef OO_RX_RING
#define OO_RX_RING 12
#define OO_RX_POLL 1
#include "oo_rx_kernel.hip"
