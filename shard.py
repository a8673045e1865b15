# SPDX-License-Identifier: BSD-2-Clause
"""How a packet stream is split across ranks (one rank per GPU).

Packets are independent and the filter table is read-only during a batch
(SURVEY.md §8(e)), so each rank owns a contiguous packet range and no
collective touches the data path.
"""


def shard_range(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """(first, count) of rank's contiguous share of n_total packets."""
    base, extra = divmod(n_total, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)
