# SPDX-License-Identifier: BSD-2-Clause
"""Phase timeline of rx_split (diagnostic; needs a -DOO_RX_STAMPS build via
OO_RX_LIB): per phase, how long streamers stream and wait at the barrier
and how long the parser finalises/parses and waits.

    OO_RX_LIB=build/var_st.so OO_RX_KERNEL=split python tools/split_stamps.py --config 2
"""
import argparse, ctypes, json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

def main():
    ap = argparse.ArgumentParser(); ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--ws", type=int, default=2)
    args = ap.parse_args()
    import torch
    from bench import DEFAULT_N
    from onload_amd import pktgen
    from onload_amd.rx import GpuRxStack
    n = DEFAULT_N[args.config]
    filters, socks = pktgen.world(args.config)
    buf, desc = pktgen.generate(args.config, n)
    g = GpuRxStack(device=0); g.load_world(filters, socks)
    lib = g._lib
    lib.oo_gpu_rx_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    fr = torch.from_numpy(buf).cuda(); de = torch.from_numpy(desc.view(np.uint8)).cuda()
    out = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    blocks = 4096; W = args.ws + 1
    st = torch.zeros(blocks * W * 64 * 8, dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    g.sync(s)
    for _ in range(3):
        g.handle_rx_batch_dev(fr.data_ptr(), fr.numel(), de.data_ptr(), n, out.data_ptr(), 0, s)
    lib.oo_gpu_rx_debug_stamps(g._ctx, ctypes.c_void_p(st.data_ptr()))
    torch.cuda.synchronize()
    g.handle_rx_batch_dev(fr.data_ptr(), fr.numel(), de.data_ptr(), n, out.data_ptr(), 0, s)
    torch.cuda.synchronize()
    a = st.cpu().numpy().reshape(blocks, W, 64, 8).astype(np.float64)
    used = a[:, 0, :, 0] != 0
    nb = int(used.any(1).sum()); K = int(used[0].sum())
    a = a[:nb]
    t0 = a[:, :, :, 0][a[:, :, :, 0] != 0].min()
    ns = 10.0
    S = a[:, :args.ws, :K]; Pp = a[:, args.ws, :K + 1]
    res = {"blocks": nb, "phases": K,
           "span_us": float((a[a != 0].max() - t0) * ns / 1e3),
           "streamer_us_per_phase": {"stream": float(((S[..., 1] - S[..., 0]) * ns).mean() / 1e3),
                                     "to_barrier": float(((S[..., 2] - S[..., 1]) * ns).mean() / 1e3),
                                     "barrier_wait": float(((S[..., 3] - S[..., 2]) * ns).mean() / 1e3)},
           "parser_us_per_phase": {"finalize": float(((Pp[:, 1:K, 1] - Pp[:, 1:K, 0]) * ns).mean() / 1e3),
                                   "parse": float(((Pp[:, :K, 2] - Pp[:, :K, 1]) * ns).mean() / 1e3),
                                   "barrier_wait": float(((Pp[:, :K, 3] - Pp[:, :K, 2]) * ns).mean() / 1e3)}}
    print(json.dumps(res))

if __name__ == "__main__":
    main()
