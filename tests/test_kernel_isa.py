# SPDX-License-Identifier: BSD-2-Clause
"""Static checks on the gfx950 code object that the kernels' counted
`s_waitcnt vmcnt(N)` waits rely on (oo_rx_kernel.hip "rx_kernel"):

* no scratch: a spill or stack object adds vector-memory operations the
  counts do not know about (they only make a wait stricter, but each costs a
  drain on the stream), so the kernels must stay within their VGPR budget;
* the stores per tile are exactly the ones the counts assume: rx_kernel two
  16-B record stores (NST), tx_kernel four 16-B granule stores plus two
  16-bit check-field stores (NST_TX), all global (a flat store counts in
  lgkmcnt too) -- a compiler that merged or split stores would make the
  waits too loose (round 1's byte stores were in fact merged).
  Besides them each kernel has one 4-B `sc1` store, before its tile loop:
  the next launch's claim counters zeroed (drained by the prologue's wait).

Compiles the kernel source to assembly with hipcc (cross-compiles, no GPU)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "onload_amd", "csrc", "oo_rx_kernel.hip")
SRC_SHORT = os.path.join(ROOT, "onload_amd", "csrc", "oo_rx_kernel_short.hip")
RX_SHORT = "_ZN11oo_rx_short9rx_kernelEN5oo_rx7KParamsE"
SRC_POLL = os.path.join(ROOT, "onload_amd", "csrc", "oo_rx_kernel_poll.hip")
RX_POLL = "_ZN10oo_rx_poll9rx_kernelEN5oo_rx8PollArgsE"
HIPCC = "/opt/rocm/bin/hipcc"


def _compile(tmp_path_factory, src):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("isa") / "k.s"
    r = subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950",
                        "--offload-device-only", "-S", "-o", str(out), src,
                        "-Rpass-analysis=kernel-resource-usage"],
                       capture_output=True, text=True, check=True)
    return out.read_text(), r.stderr


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    return _compile(tmp_path_factory, SRC)


@pytest.fixture(scope="module")
def asm_short(tmp_path_factory):
    """The short-frame rx_kernel (2-slot ring, oo_rx_kernel_short.hip)."""
    return _compile(tmp_path_factory, SRC_SHORT)


def _body(text, name):
    m = re.search(rf"^{name}:.*?^\.Lfunc_end", text, re.S | re.M)
    assert m, name
    return m.group(0)


def _usage(stderr, mangled):
    i = stderr.index(f"Function Name: {mangled}")
    block = stderr[i:i + 2000]
    get = lambda k: int(re.search(rf"{k}: (\d+)", block).group(1))  # noqa: E731
    return {k: get(k) for k in ("VGPRs", "ScratchSize \\[bytes/lane\\]", "VGPRs Spill")}


@pytest.mark.parametrize("kernel", ["_ZN5oo_rx9rx_kernelENS_7KParamsE",
                                    "_ZN5oo_rx9tx_kernelENS_7KParamsE"])
def test_no_scratch(asm, kernel):
    text, stderr = asm
    u = _usage(stderr, kernel)
    assert u["VGPRs Spill"] == 0, u
    # no scratch access in the kernel or the (rare-path) function it calls; the
    # reported ScratchSize may still hold a call frame reservation
    assert "scratch_" not in _body(text, kernel)
    assert "scratch_" not in _body(text, "_ZN5oo_rx17window_sum_globalEmii")
    assert u["VGPRs"] <= 168, u  # 3 waves per SIMD (amdgpu_waves_per_eu(3))


def test_store_counts(asm):
    text, _ = asm
    rx = _body(text, "_ZN5oo_rx9rx_kernelENS_7KParamsE")
    # store_records: two 16-B stores per tile (NST)
    assert len(re.findall(r"global_store_dwordx4", rx)) == 2
    assert not re.findall(r"global_store_(byte|short|dwordx2)", rx)
    # zero_claim_set: the next launch's claim set, three `sc1` stores
    assert len(re.findall(r"global_store_dword .* sc1$", rx, re.M)) == 3
    assert len(re.findall(r"global_store_dword\b", rx)) == 3
    tx = _body(text, "_ZN5oo_rx9tx_kernelENS_7KParamsE")
    assert len(re.findall(r"global_store_short\b", tx)) == 2
    assert len(re.findall(r"global_store_dwordx4", tx)) == 4
    assert not re.findall(r"global_store_(byte|dwordx2)", tx)
    assert len(re.findall(r"global_store_dword\b", tx)) == 3
    for body in (rx, tx):  # flat stores would count in lgkmcnt as well
        assert not re.findall(r"flat_store|flat_load|flat_atomic", body)


def test_short_kernel_same_invariants(asm_short):
    text, stderr = asm_short
    u = _usage(stderr, RX_SHORT)
    assert u["VGPRs Spill"] == 0, u
    assert u["VGPRs"] <= 168, u
    rx = _body(text, RX_SHORT)
    assert "scratch_" not in rx
    assert len(re.findall(r"global_store_dwordx4", rx)) == 2
    assert not re.findall(r"global_store_(byte|short|dwordx2)", rx)
    assert len(re.findall(r"global_store_dword\b", rx)) == 3  # zero_claim_set
    assert not re.findall(r"flat_store|flat_load|flat_atomic", rx)


@pytest.fixture(scope="module")
def asm_poll(tmp_path_factory):
    """The poll instance (12-slot ring, oo_rx_kernel_poll.hip)."""
    return _compile(tmp_path_factory, SRC_POLL)


def test_poll_kernel_same_invariants(asm_poll):
    """The poll instance: no scratch and the same stores per tile; besides
    zero_claim_set's three, one more 4-B `sc0 sc1` store -- the done word,
    after the wave's last wait -- and the one returning system-scope add
    that counts the wave out (oo_rx_kernel.hip "The poll instance")."""
    text, stderr = asm_poll
    u = _usage(stderr, RX_POLL)
    assert u["VGPRs Spill"] == 0, u
    assert u["VGPRs"] <= 256, u
    rx = _body(text, RX_POLL)
    assert "scratch_" not in rx
    assert len(re.findall(r"global_store_dwordx4", rx)) == 2
    assert not re.findall(r"global_store_(byte|short|dwordx2)", rx)
    assert len(re.findall(r"global_store_dword\b", rx)) == 4
    assert len(re.findall(r"global_store_dword .* sc0 sc1$", rx, re.M)) == 1
    assert len(re.findall(r"global_atomic_add .* sc0 sc1$", rx, re.M)) == 1
    assert not re.findall(r"flat_store|flat_load|flat_atomic", rx)
    # the kernel holds rx_kernel alone
    assert "tx_kernel" not in text and "win_kernel" not in text


WIN = "_ZN5oo_rx10win_kernelENS_7KParamsE"
BODY = "_ZN5oo_rx11body_kernelENS_7KParamsE"


def _lds(stderr, mangled):
    i = stderr.index(f"Function Name: {mangled}")
    return int(re.search(r"LDS Size \[bytes/block\]: (\d+)", stderr[i:i + 2000]).group(1))


def test_split_kernels_no_scratch(asm):
    """The split transform (win_kernel, body_kernel): no spill -- a reload in
    the tile loop would wait for the staged next tile's windows -- and
    win_kernel fits twelve waves per CU (168 VGPRs; 10 KiB of LDS a wave plus
    the block's bitmap copy, three 4-wave blocks)."""
    text, stderr = asm
    for k in (WIN, BODY):
        u = _usage(stderr, k)
        assert u["VGPRs Spill"] == 0, (k, u)
        assert "scratch_" not in _body(text, k), k
    assert _usage(stderr, WIN)["VGPRs"] <= 168
    assert 3 * _lds(stderr, WIN) <= 160 * 1024
    assert _usage(stderr, BODY)["VGPRs"] <= 128


def test_gseq_body_kernel_no_scratch(asm_short):
    """body_kernel with per-group job sequences (the short-frame instance)."""
    text, stderr = asm_short
    k = "_ZN11oo_rx_short11body_kernelEN5oo_rx7KParamsE"
    u = _usage(stderr, k)
    assert u["VGPRs Spill"] == 0, u
    assert "scratch_" not in _body(text, k)
    assert not re.findall(r"flat_store|flat_load|flat_atomic", _body(text, k))


def test_split_store_counts(asm):
    text, _ = asm
    w = _body(text, WIN)
    # store_records (NST = 2), the pending word, and the sc1 stores: three in
    # zero_claim_set plus the body flag
    assert len(re.findall(r"global_store_dwordx4", w)) == 2
    assert len(re.findall(r"global_store_dwordx2", w)) == 1
    assert len(re.findall(r"global_store_dword .* sc1$", w, re.M)) == 4
    assert len(re.findall(r"global_store_dword\b", w)) == 4
    assert not re.findall(r"global_store_(byte|short)", w)
    for k in (WIN, BODY):
        assert not re.findall(r"flat_store|flat_load|flat_atomic", _body(text, k)), k


def test_win_kernel_counted_wait_after_staging(asm):
    """window_loop stages the next tile inside the demux (oo_rx_kernel.hip
    kx_lookup, `issued`): the key index's first-level loads are untracked and
    one counted `s_waitcnt vmcnt(HC + 2)` (the inline-asm vm_wait) after the
    staging covers them.  That holds only if every path from those loads to
    the wait issues exactly HC + 2 = 10 vector-memory operations -- the
    descriptor line, one of the two staging forms (all rows, or masked rows:
    eight LDS-DMA rows each), the claim.  (A compiler wait in between only
    makes the counted one redundant.)"""
    text, _ = asm
    win = _body(text, WIN).splitlines()
    sites = [i for i, l in enumerate(win)
             if re.search(r"s_waitcnt vmcnt\(10\)", l) and "ASMSTART" in win[i - 1]]
    assert sites, "no counted wait after the staging"
    for w in sites:
        i, lds, other = w - 2, 0, []
        while not re.match(r"^\s*global_load_dwordx4 v\[\d+:\d+\], v\[\d+:\d+\], off$", win[i]):
            if "global_load_lds" in win[i]:
                lds += 1
            elif re.match(r"^\s*(global_|buffer_|scratch_|flat_)", win[i]):
                other.append(win[i].split()[0])
            i -= 1
            assert i >= 0, "no untracked load before the counted wait"
        # the descriptor line and the two staging forms laid out one after
        # the other, then the claim
        assert lds == 1 + 8 + 8 and other == ["global_atomic_add"], (w, lds, other)
