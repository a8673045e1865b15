# SPDX-License-Identifier: BSD-2-Clause
"""The one-rank RCCL group cases of test_gpu_group_rccl.py, each run as a
child process (python rccl_one_rank.py every_leg|bad_count): prints
"ok <case>" when the case passed, raises otherwise."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from onload_amd import _abi, pktgen  # noqa: E402
from onload_amd.group import GpuRxGroup  # noqa: E402
from oracle_lib import OracleStack, counters_of  # noqa: E402  (the checker only)


def every_leg(torch):
    config, n = 5, 40000
    filters, socks = pktgen.world(config)
    g = GpuRxGroup.join(0, 0, 1, GpuRxGroup.rccl_id())
    assert g.uses_rccl and g.rank == 0
    g.load_world(filters, socks)
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    queued = len(filters) + len(socks)
    assert queued > 8192  # more than one broadcast chunk
    assert g.share_ops(sh) == queued
    assert g.share_ops(sh) == 0  # the queue was emptied
    g.share_tables(sh)
    m = g.members[0]
    buf, desc = pktgen.generate(config, n)
    frames = torch.from_numpy(buf).cuda()
    d_desc = torch.from_numpy(desc.view(np.uint8)).cuda()
    out = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    ctr = torch.zeros(32, dtype=torch.int32, device="cuda")
    m.sync(sh)
    m.handle_rx_batch_dev(frames.data_ptr(), frames.numel(), d_desc.data_ptr(), n,
                          out.data_ptr(), ctr.data_ptr(), sh)
    g.sum_counters(ctr.data_ptr(), sh)
    dst = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    g.gather_rccl(out.data_ptr(), n, dst.data_ptr(), [n], sh)
    torch.cuda.synchronize()
    o = OracleStack()
    o.load_world(filters, socks)
    want = o.handle_rx_batch(buf, desc, nthreads=8)
    got = dst.cpu().numpy().view(_abi.RESULT_DTYPE)
    assert got.tobytes() == want.tobytes()
    assert (ctr.cpu().numpy().view(np.uint32)[:len(counters_of(want))] == counters_of(want)).all()
    # a change after the image: queued, shared, the batch sees it
    f = filters[0]
    ra = None if f.raddr_any else bytes(f.raddr)[: 4 if f.af == 4 else 16]
    la = bytes(f.laddr)[: 4 if f.af == 4 else 16]
    assert g.filter_remove_raw(f.sock, f.af, la, f.lport_be, ra, f.rport_be, f.proto) == 0
    assert g.share_ops(sh) == 1
    torch.cuda.synchronize()
    g.close()


def bad_count(torch):
    g = GpuRxGroup.join(0, 0, 1, GpuRxGroup.rccl_id())
    out = torch.zeros(64 * 32, dtype=torch.uint8, device="cuda")
    dst = torch.zeros(64 * 32, dtype=torch.uint8, device="cuda")
    try:
        g.gather_rccl(out.data_ptr(), 64, dst.data_ptr(), [63], 0)
    except OSError:
        pass
    else:
        raise AssertionError("a gather of 63 records for 64 was accepted")
    g.close()


def main():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    case = sys.argv[1]
    {"every_leg": every_leg, "bad_count": bad_count}[case](torch)
    torch.cuda.synchronize()
    print(f"ok {case}", flush=True)


if __name__ == "__main__":
    main()
