"""Set-up of the one-shot xGMI all-reduce (``fedmi/ops/csrc/peer_allreduce.hip``).

The fused round engine's FedAvg message is ~50 KB (the reference MLP's parameter image plus
metric tails), so its all-reduce is latency-bound.  On an MI355X node every GPU has a direct
xGMI link to each of its 7 peers: the native ``PeerAllReduce`` maps every rank's send buffers
through HIP IPC and reduces them in ONE kernel (publish flag -> wait -> pull all peers over
the 7 links at once -> sum in rank order), instead of a ring's 2 x 7 dependent steps.  RCCL
stays the path for bandwidth-bound messages (the wide-MLP buckets) and the fallback here.

:func:`make_peer_allreduce` is collective: every rank either gets a working, self-tested
communicator or ``None`` -- never a mix, so ranks cannot disagree about the data plane.
"""
from __future__ import annotations

import os
import sys
import threading
import weakref
from typing import Optional

import numpy as np
import torch

PEER_MAX_WORLD = 8


def _all_ok(comm, ok: bool) -> bool:
    """Logical AND over ranks (host control plane)."""
    return all(comm.allgather(bool(ok)))


def fill_values(n: int, rank: int, salt: int) -> np.ndarray:
    """Host copy of the self-test payload written by ``fill_test`` (peer_fill_kernel)."""
    i = np.arange(n, dtype=np.uint64)
    h = (i * np.uint64(2654435761) + np.uint64(rank * 40503) + np.uint64(salt * 97)) & np.uint64(0xFFFFFFFF)
    return (h % np.uint64(2048)).astype(np.float64) * 0.25 - 256.0


def selftest(h, comm, device, calls: int = 4, timeout_s: float = 10.0) -> bool:
    """Run ``calls`` all-reduces of a known payload (both parities) and check every float on
    every rank.  All ranks run every call even after a mismatch, so nobody is left waiting."""
    n = int(h.n_floats)
    out = torch.empty(n, dtype=torch.float32, device=device)
    s = torch.cuda.current_stream(device)
    h.set_timeout(timeout_s)
    ok = True
    for k in range(calls):
        salt = 1000 + k
        h.fill_test(k & 1, salt, s.cuda_stream)
        h.allreduce(k & 1, out.data_ptr(), s.cuda_stream)
        got = out.cpu().numpy()
        expect = sum(fill_values(n, r, salt) for r in range(comm.size)).astype(np.float32)
        ok = ok and bool(np.array_equal(got, expect))
    # the Adam-fused chunk exchange (peer_device.h): same payload, chunk flags, both parities
    nc = int(getattr(h, "n_chunks", 0))
    if nc > 0:
        m = min(n, nc * 64)
        out.zero_()
        for k in range(2):
            salt = 2000 + k
            h.fill_test(k & 1, salt, s.cuda_stream)
            h.chunk_test(k & 1, k + 1, out.data_ptr(), s.cuda_stream)
            got = out.cpu().numpy()[:m]
            expect = sum(fill_values(n, r, salt) for r in range(comm.size)).astype(np.float32)[:m]
            ok = ok and bool(np.array_equal(got, expect))
            comm.Barrier()  # every rank has read this parity before it is refilled
        # LL weight chunks (peer_device.h): values pushed with the call index, both parities
        if bool(getattr(h, "uses_ll", False)):
            for k in range(2):
                salt, target = 3000 + k, 3 + k
                out.zero_()
                h.fill_test(target & 1, salt, s.cuda_stream)
                comm.Barrier()  # every rank's payload is in place before anyone pushes it
                h.ll_test(target, out.data_ptr(), s.cuda_stream)
                got = out.cpu().numpy()[:m]
                expect = sum(fill_values(n, r, salt) for r in range(comm.size)).astype(np.float32)[:m]
                ok = ok and bool(np.array_equal(got, expect))
            # RS+AG weight chunks (peer_device.h peer_rsag): owner sums, then pushes the sums back
            if bool(getattr(h, "uses_rsag", False)):
                for k in range(2):
                    salt, target = 4000 + k, 5 + k
                    out.zero_()
                    h.fill_test(target & 1, salt, s.cuda_stream)
                    comm.Barrier()
                    h.rsag_test(target, out.data_ptr(), s.cuda_stream)
                    got = out.cpu().numpy()[:m]
                    expect = sum(fill_values(n, r, salt) for r in range(comm.size)).astype(np.float32)[:m]
                    ok = ok and bool(np.array_equal(got, expect))
    ok = ok and h.error() == 0
    return ok


# The exchanging Adam kernels are 1024-thread workgroups at ~125 VGPRs: one resident workgroup
# per CU.  The spinning grids of every rank sharing a GPU must be resident together, so the slot
# count is the device's CU count (MI355X: 256; fewer on a partitioned device or another SKU).
ADAM_WORKGROUPS_PER_CU = 1
SHARED_GPU_ADAM_SLOTS = 256   # MI355X default when the device cannot be queried


def adam_slots(device=None) -> int:
    """Adam workgroups that can be resident at once on ``device`` (CUs x workgroups per CU)."""
    if device is not None and torch.cuda.is_available():
        try:
            return int(torch.cuda.get_device_properties(torch.device(device)).multi_processor_count) \
                * ADAM_WORKGROUPS_PER_CU
        except Exception:  # noqa: BLE001 -- fall back to the MI355X figure
            pass
    return SHARED_GPU_ADAM_SLOTS


def device_key(device) -> str:
    """Identity of the physical GPU behind ``device`` (same string in every process that uses it)."""
    p = torch.cuda.get_device_properties(torch.device(device))
    uuid = getattr(p, "uuid", None)
    if uuid is not None:
        return str(uuid)
    return f"{getattr(p, 'pci_domain_id', 0)}:{getattr(p, 'pci_bus_id', 0)}:{getattr(p, 'pci_device_id', 0)}"


def shared_adam_grid(n_sharing: int, adam_blocks: int, slots: int = SHARED_GPU_ADAM_SLOTS) -> int:
    """Workgroups of the LL Adam kernel when ``n_sharing`` exchanging ranks sit on ONE GPU
    with ``slots`` resident Adam workgroups (:func:`adam_slots`; 0 = the full grid of
    ``adam_blocks``).  Every Adam block spins until the same block of every rank has pushed its
    chunk, so all ranks' blocks must be co-resident; when the full grids cannot be, each rank
    walks its blocks on (slots / 2) / n_sharing workgroups -- half the device, so the ranks'
    train kernels keep room -- (fl_adam_ll_grid_kernel for LL chunks, fl_adam_grid_kernel for
    publish / wait / pull; bit-identical)."""
    if n_sharing < 2 or n_sharing * adam_blocks <= slots:
        return 0
    return max(1, (slots // 2) // n_sharing)


DEFAULT_PEER_TIMEOUT_S = 60.0


def peer_timeout_s(timeout_s: Optional[float] = None) -> float:
    """Seconds a device wait of the xGMI plane waits for a peer before it reports the peer as
    failed to every rank: ``timeout_s``, else ``$FEDMI_PEER_TIMEOUT_S``, else 60."""
    if timeout_s is not None:
        return float(timeout_s)
    env = os.environ.get("FEDMI_PEER_TIMEOUT_S", "").strip()
    return float(env) if env else DEFAULT_PEER_TIMEOUT_S


# Live communicators of this process: Comm.Abort / watchdogs release their spinning kernels and
# tell every peer (abort_all) before the process exits.
_LIVE = weakref.WeakSet()


def abort_all(wait_s: float = 1.0) -> int:
    """Fail-fast abort of every live xGMI communicator of this process: the host abort word
    ends this rank's device waits and every rank's failure word is written, so the peers stop
    waiting at once (reference: any failure -> comm.Abort(),
    FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py:203-205).  Runs on a helper thread
    bounded by ``wait_s`` per communicator (a wedged runtime must not keep the process alive).
    Returns the number of communicators whose peers were told in time."""
    told = []
    for h in list(_LIVE):
        res = []
        t = threading.Thread(target=lambda: res.append(bool(h.abort(wait_s))), daemon=True)
        t.start()
        t.join(wait_s + 1.0)
        told.append(bool(res and res[0]))
    return sum(told)


# Communicators whose engine is gone.  A rank's send buffers, flags and ring are READ BY ITS
# PEERS, so a rank must not free them when its own engine is dropped: a slower peer may still be
# pulling its last round's tails (freed memory reused by the next allocation reads as zeros there).
# retire() parks the communicator; the next collective set-up frees it once every rank has
# arrived there with its device work drained (make_peer_allreduce), i.e. past its last read.
_RETIRED = []


def retire(h) -> None:
    """Park a communicator whose owner is done with it (see _RETIRED); no collective needed."""
    if h is not None:
        _RETIRED.append(h)


def _free_retired() -> None:
    while _RETIRED:
        try:
            _RETIRED.pop().close()
        except Exception:  # noqa: BLE001 -- best effort: the process keeps working either way
            pass


def _test_fail_ranks() -> set:
    """Test knob ``FEDMI_TEST_PEER_FAIL=1,3``: the peer set-up fails on these ranks (exercises
    the agreed fallback of every rank to the next data plane)."""
    env = os.environ.get("FEDMI_TEST_PEER_FAIL", "").strip()
    return {int(x) for x in env.split(",") if x.strip() != ""}


def make_peer_allreduce(comm, n_floats: int, device, timeout_s: Optional[float] = None, check: bool = True,
                        n_chunks: int = 0):
    """Collective.  Returns a native ``PeerAllReduce`` of ``n_floats`` floats, open and
    self-tested on every rank, or ``None`` on every rank (then the caller uses RCCL).
    ``n_chunks``: chunk-flag table for the Adam-fused exchange of the round engine.
    ``timeout_s``: see :func:`peer_timeout_s`."""
    from ..ops import native
    if comm is None or comm.size < 2 or comm.size > PEER_MAX_WORLD:
        return None
    timeout_s = peer_timeout_s(timeout_s)
    m = native()
    # this rank's device work (incl. reads of retired peers' buffers) is done before it reports
    # in below; once every rank has reported, every retired communicator is past its last use
    torch.cuda.synchronize(torch.device(device))
    h, why = None, ""
    try:
        if comm.rank in _test_fail_ranks():
            raise RuntimeError("peer set-up failed (FEDMI_TEST_PEER_FAIL)")
        h = m.PeerAllReduce(comm.size, comm.rank, torch.device(device).index or 0, int(n_floats), float(timeout_s),
                            int(n_chunks))
        handle = bytes(h.handle())
    except Exception as e:  # noqa: BLE001 -- reported, and every rank falls back together
        handle, why = None, f"rank {comm.rank}: {e}"
    gathered = comm.allgather((handle, device_key(device)))
    _free_retired()
    handles = [g[0] for g in gathered]
    ok = all(x is not None for x in handles)
    if ok and n_chunks > 0:
        # ranks sharing this rank's GPU (tests, bench --share-gpu): bound the spinning Adam grid
        env = os.environ.get("FEDMI_ADAM_GRID", "")
        if env == "":
            mine = gathered[comm.rank][1]
            h.adam_grid = shared_adam_grid(sum(g[1] == mine for g in gathered), n_chunks - 1, adam_slots(device))
    if ok:
        try:
            h.open(handles)
        except Exception as e:  # noqa: BLE001
            ok, why = False, f"rank {comm.rank}: {e}"
    ok = _all_ok(comm, ok)
    if ok and check:
        ok = _all_ok(comm, selftest(h, comm, device))
        why = why or "self-test mismatch or timeout"
    if h is not None:
        h.set_timeout(timeout_s)
    if not ok:
        # every rank prints its own reason (the failing rank knows why; the others only that it failed)
        print(f"[fedmi] rank {comm.rank}: one-shot xGMI all-reduce unavailable ({why or 'peer set-up failed on another rank'}); "
              "falling back to the next data plane", file=sys.stderr, flush=True)
        comm.Barrier()  # nobody still reads a buffer we are about to free
        if h is not None:
            h.close()
        return None
    # The self-test left its payload in the send buffers; the engine never writes the image
    # padding, which must read as 0.  Every rank finished its self-test reads before the
    # allgather above, so the buffers can be zeroed now; the barrier orders the zeroing
    # before any rank's first real call.
    h.clear()
    comm.Barrier()
    _LIVE.add(h)
    return h


_TEST_ERROR_FIRED = False


class PeerFailure(RuntimeError):
    """A rank of the xGMI data plane failed (timed out waiting for a peer, or aborted)."""


def describe_peer_error(word: int, timeout_s: Optional[float] = None) -> str:
    """Human-readable form of the sticky failure word (peer_device.h PEER_ERR_*)."""
    kind, who, missing = (word >> 16) & 0xFF, (word >> 8) & 0xFF, word & 0xFF
    if kind == 2:
        return f"rank {who} aborted the job"
    if kind == 1:
        t = f" {timeout_s:g} s" if timeout_s else " its timeout"
        if missing == 0xFE:
            return f"rank {who}: its own evaluation blocks did not finish within{t}"
        return f"rank {who} waited{t} for rank {missing}, which died or stalled"
    return f"failure word {word:#x}"


def check_peer_error(h) -> None:
    """Raise :class:`PeerFailure` if any rank reported a failure on this communicator: the
    rounds since then were aggregated from missing contributions and are invalid."""
    if h is None:
        return
    word = int(h.error())
    global _TEST_ERROR_FIRED
    if not word and not _TEST_ERROR_FIRED and os.environ.get("FEDMI_TEST_PEER_ERROR", "") == "1":
        _TEST_ERROR_FIRED = True   # test knob: one simulated failure report per process (every rank alike)
        word = (1 << 16) | (0xFF << 8) | 0xFF
    if word:
        raise PeerFailure("xGMI data plane failed: " + describe_peer_error(word, getattr(h, "timeout_s", None))
                          + "; rounds since then are invalid")
