// SPDX-License-Identifier: BSD-2-Clause
// Prints oo_rx_device.h's kx_hash for the ten-word keys read from stdin
// (one key per line, decimal words), so tests/test_kx_hash.py can check the
// Python restatement the collision tests build their keys with.
#include <cstdio>

#include "../../onload_amd/csrc/oo_rx_device.h"

int main() {
  unsigned w[10];
  while (std::scanf("%u %u %u %u %u %u %u %u %u %u", &w[0], &w[1], &w[2], &w[3], &w[4], &w[5],
                    &w[6], &w[7], &w[8], &w[9]) == 10)
    std::printf("%u\n", oo_rx::kx_hash(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7], w[8], w[9]));
  return 0;
}
