"""Process-group runtime: one process per GPU (= one federated client).

The reference talks MPI through mpi4py's pickle collectives on ``MPI.COMM_WORLD``
(``FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py:212-214``; every call site in
SURVEY §2.4).  :class:`Comm` keeps that object API -- ``Get_rank``, ``Get_size``,
``gather``, ``bcast``, ``Barrier``, ``Abort`` -- so reference-style driver code keeps
working, but the data plane is different:

* **control plane** (rare, host objects: start-up checks, final reports): gloo via
  ``torch.distributed``;
* **data plane** (every round, device buffers): one in-place SUM all-reduce on a flat
  device buffer.  Backends:

  - ``xgmi``  -- (default on GPUs) the fused round engine aggregates with the one-shot
    peer all-reduce over xGMI (``fedmi.parallel.peer``: IPC-mapped send buffers, one kernel
    per round, self-tested at start-up); everything else uses the RCCL communicator below,
    which is also the automatic fallback.
  - ``rccl``  -- the engine-owned RCCL communicator in the native extension
    (``RcclComm``: ``ncclCommInitRank`` over xGMI, unique id exchanged over the gloo
    store).  The engine issues ``ncclAllReduce`` itself, inside captured HIP graphs.
  - ``nccl``  -- torch's ProcessGroupNCCL (which *is* RCCL on ROCm), for callers that
    want torch to own the communicator.
  - ``gloo``  -- CPU tensors (BASELINE config 1: "2-client FedAvg ... CPU + gloo").

Launch with ``torchrun --nproc-per-node N --master-addr 127.0.0.1 ...`` or, like the reference,
``mpiexec -n N python ...`` (Open MPI / MPICH environments are recognised,
:func:`launch_env`); the node-local rank selects the device (fixes the reference's
everyone-on-GPU-0).
"""
from __future__ import annotations

import contextlib
import os
import sys
import time
from typing import Any, List, Optional

import torch
import torch.distributed as dist


def _env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


# Rank / size / node-local rank as set by the launcher that started this process: torchrun, or
# the MPI launchers the reference is run with (``mpiexec -n k python <script>``, SURVEY §1 L0 --
# Open MPI's and MPICH/Hydra's per-process environment).  mpi4py is not needed: the control
# plane is gloo over a TCP store, so an MPI launch only has to tell every process who it is.
# (Allocation-wide variables such as Slurm's SLURM_NTASKS are deliberately not read: they are
# also set for a process started alone inside the allocation, which would then wait for peers.)
_LAUNCH_VARS = (
    ("RANK", "WORLD_SIZE", "LOCAL_RANK"),                                              # torchrun
    ("OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_RANK"),    # Open MPI
    ("PMI_RANK", "PMI_SIZE", "MPI_LOCALRANKID"),                                       # MPICH / Hydra
)


def launch_env() -> tuple:
    """``(rank, world_size, local_rank, launcher)`` of this process (``(0, 1, 0, None)`` when
    started alone).  The first launcher whose rank and size variables are both set wins; a
    missing local rank defaults to the rank (one node)."""
    for i, (r, n, lr) in enumerate(_LAUNCH_VARS):
        if os.environ.get(r, "") != "" and os.environ.get(n, "") != "":
            rank, size = _env_int(r, 0), _env_int(n, 1)
            return rank, size, _env_int(lr, rank), ("torchrun", "openmpi", "mpich")[i]
    return 0, 1, 0, None


DATA_PLANES = ("xgmi", "rccl", "nccl")


def resolve_backend(backend: str, device_type: str) -> str:
    """``auto`` -> gloo on CPU; on GPUs ``$FEDMI_DATA_PLANE`` (xgmi | rccl | nccl, default
    xgmi), so a launcher can A/B the FedAvg data planes without touching the command line."""
    if backend != "auto":
        return backend
    if device_type != "cuda":
        return "gloo"
    plane = os.environ.get("FEDMI_DATA_PLANE", "xgmi").strip().lower() or "xgmi"
    if plane not in DATA_PLANES:
        raise ValueError(f"FEDMI_DATA_PLANE={plane!r}: expected one of {DATA_PLANES}")
    return plane



@contextlib.contextmanager
def _c_stdout_to_stderr():
    """File descriptor 1 -> 2 for the duration (output of native libraries included)."""
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)

RCCL_ALGO_DEFAULT = "Ring"


def pin_rccl_env(proto: str) -> dict:
    """Pin RCCL's algorithm and protocol for reproducible collectives and return
    what this process's communicators will use.  RCCL reads them when a communicator is
    created, so this runs before ``ncclCommInitRank`` / the nccl process group.  Values the
    user exported win.  Defaults: Ring (xGMI is point-to-point; every rank on one ring over its
    direct links) with the protocol of the messages this process sends -- LL for the
    latency-bound FedAvg images of the fused engine (45 KB - 1 MB), Simple for the wide
    MLP's bandwidth-bound per-layer buckets (16-67 MB)."""
    os.environ.setdefault("NCCL_ALGO", RCCL_ALGO_DEFAULT)
    os.environ.setdefault("NCCL_PROTO", proto)
    return {"NCCL_ALGO": os.environ["NCCL_ALGO"], "NCCL_PROTO": os.environ["NCCL_PROTO"]}


class Comm:
    """``rccl=False`` (with ``backend='xgmi'``) forbids the RCCL communicator: device
    all-reduces outside the round engine then go through the host.  That is the setting for
    several ranks sharing one GPU (tests), which RCCL does not support.  ``rccl_proto``: the
    RCCL protocol pinned for this process (:func:`pin_rccl_env`; reported as ``rccl_env``).
    ``rccl_timeout_s`` (or ``$FEDMI_RCCL_TIMEOUT_S``) bounds the RCCL bootstrap (:meth:`rccl`)."""

    def __init__(self, backend: str = "auto", device: Optional[str] = None, timeout_s: float = 600.0,
                 rccl: bool = True, rccl_proto: str = "LL", rccl_timeout_s: float = 120.0):
        self.rank, self.size, self.local_rank, self.launcher = launch_env()
        if device is None or device == "auto":
            device = "cuda" if torch.cuda.is_available() else "cpu"
        if device.startswith("cuda"):
            idx = self.local_rank if device == "cuda" else int(device.split(":")[1])
            torch.cuda.set_device(idx)
            self.device = torch.device("cuda", idx)
        else:
            self.device = torch.device("cpu")
        backend = resolve_backend(backend, self.device.type)
        if backend not in ("xgmi", "rccl", "nccl", "gloo"):
            raise ValueError(f"unknown backend {backend!r}")
        if self.device.type == "cpu" and backend != "gloo":
            raise ValueError(f"backend {backend!r} needs a GPU device")
        self.backend = backend
        self.peer_allreduce = backend == "xgmi"   # round engines use the one-shot xGMI all-reduce
        self.native = None       # RcclComm
        self.rccl_env = None     # pinned NCCL_ALGO / NCCL_PROTO when an RCCL communicator exists
        self._nccl_group = None
        self._initialized_here = False
        self.rccl_allowed = backend == "rccl" or (backend == "xgmi" and rccl)
        self.rccl_proto = rccl_proto
        self.rccl_timeout_s = float(os.environ.get("FEDMI_RCCL_TIMEOUT_S", "") or rccl_timeout_s)
        self._rccl_factory = None  # tests inject a fake bootstrap (CPU); None -> native RcclComm
        self.rccl_error = None     # why RCCL was disabled after a failed bootstrap (rccl_or_host)
        self._agree_gen = 0
        if self.size > 1:
            if not dist.is_initialized():
                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                os.environ.setdefault("MASTER_PORT", "29500")
                from datetime import timedelta
                # gloo prints its connection report on the C-level stdout; send it to stderr so
                # rank 0's stdout carries only the program's own output (bench.py's JSON line)
                with _c_stdout_to_stderr():
                    dist.init_process_group("gloo", rank=self.rank, world_size=self.size,
                                            timeout=timedelta(seconds=timeout_s))
                self._initialized_here = True
            if backend in ("rccl", "nccl"):
                self.rccl_env = pin_rccl_env(rccl_proto)
            if backend == "rccl":
                self.rccl()  # the data plane IS the communicator: bootstrap it now (bounded)
            elif backend == "nccl":
                self._nccl_group = dist.new_group(backend="nccl")
            # backend "xgmi": the fused engine's data plane is the peer kernel, which needs no
            # RCCL.  The communicator is created LAZILY (rccl()) by the callers that need one:
            # an engine whose peer set-up fell back, the wide MLP's buckets, sweeps, [S]/[H].

    # ---- bounded, agreed collective set-up over the gloo store ----
    def _store(self):
        return dist.distributed_c10d._get_default_store()

    def agree(self, tag: str, payload: str, timeout_s: float) -> List[str]:
        """Every rank posts ``payload`` under a fresh key and waits (at most ``timeout_s``) for
        every other rank's.  Returns the payloads in rank order; raises ``TimeoutError`` naming
        the ranks that never posted (died, or stuck before this point) instead of blocking in a
        gloo collective for the process group's whole timeout."""
        if self.size == 1:
            return [payload]
        self._agree_gen += 1
        base = f"fedmi/agree/{tag}/{self._agree_gen}/"
        store = self._store()
        store.set(base + str(self.rank), payload)
        keys = [base + str(r) for r in range(self.size)]
        t_end = time.monotonic() + float(timeout_s)
        while True:
            missing = [r for r, k in enumerate(keys) if not store.check([k])]
            if not missing:
                break
            if time.monotonic() >= t_end:
                raise TimeoutError(f"[fedmi] {tag}: rank(s) {missing} did not report within {timeout_s:g} s "
                                   f"(died or stuck before the {tag} step)")
            time.sleep(0.005)
        return [store.get(k).decode() for k in keys]

    def _share_bytes(self, tag: str, data: Optional[bytes], root: int, timeout_s: float) -> bytes:
        """Root publishes ``data`` in the store; the others wait for it, bounded."""
        self._agree_gen += 1
        key = f"fedmi/share/{tag}/{self._agree_gen}"
        store = self._store()
        if self.rank == root:
            store.set(key, data)
            return data
        t_end = time.monotonic() + float(timeout_s)
        while not store.check([key]):
            if time.monotonic() >= t_end:
                raise TimeoutError(f"[fedmi] {tag}: rank {root} did not publish within {timeout_s:g} s")
            time.sleep(0.005)
        return store.get(key)

    def rccl(self):
        """The RCCL communicator of this process, created on first use.  COLLECTIVE on first use:
        every rank must call it at the same point (SPMD).  ``None`` when RCCL is not allowed
        (``rccl=False``, e.g. ranks sharing one GPU; the caller then goes through the host).

        Set-up is bounded and agreed: the unique id travels through the gloo store with a
        deadline, the native init is non-blocking with a deadline (``RcclComm``: abort on
        timeout, GIL released), and every rank then posts its outcome and waits for everyone
        else's -- so the job either has a communicator on every rank or raises on every rank
        with the failing ranks named; never a split state, never an unbounded hang."""
        if self.native is not None or self.size == 1 or not self.rccl_allowed:
            return self.native
        t = self.rccl_timeout_s
        if self.device.type == "cuda" and self._rccl_factory is None:
            # ranks sharing a GPU (--device cuda:0 on a one-GPU box): RCCL refuses duplicate
            # devices, so every rank agrees to stay on the host path instead of failing the job
            from .peer import device_key
            keys = self.agree("rccl-devices", device_key(self.device), t)
            if len(set(keys)) < len(keys):
                self.rccl_allowed = False
                return None
        if self.rccl_env is None:
            self.rccl_env = pin_rccl_env(self.rccl_proto)
        factory = self._rccl_factory
        if factory is None:
            from ..ops import native
            m = native()
            unique_id = m.RcclComm.unique_id

            def factory(uid):
                return m.RcclComm(self.size, self.rank, uid, self.device.index, t)
        else:
            unique_id = factory.unique_id
        uid = self._share_bytes("rccl-uid", unique_id() if self.rank == 0 else None, 0, t)
        h, err = None, ""
        try:
            if str(self.rank) in os.environ.get("FEDMI_TEST_RCCL_FAIL", "").split(","):
                raise RuntimeError("RCCL bootstrap failed (FEDMI_TEST_RCCL_FAIL)")   # test knob
            h = factory(uid)
        except Exception as e:  # noqa: BLE001 -- agreed below, raised on every rank
            err = str(e).replace("\n", " ") or type(e).__name__
        try:
            outcome = self.agree("rccl-bootstrap", "ok" if h is not None else "fail:" + err, t)
        except TimeoutError as e:
            if h is not None:
                h.abort()
            raise RuntimeError(f"RCCL bootstrap not agreed: {e}") from None
        bad = [f"rank {r}: {o[5:]}" for r, o in enumerate(outcome) if o != "ok"]
        if bad:
            if h is not None:
                h.abort()
            raise RuntimeError("RCCL bootstrap failed on " + "; ".join(bad))
        self.native = h
        return h

    # ---- mpi4py-compatible object API (reference call sites) ----
    def Get_rank(self) -> int:
        return self.rank

    def Get_size(self) -> int:
        return self.size

    def gather(self, obj: Any, root: int = 0) -> Optional[List[Any]]:
        if self.size == 1:
            return [obj]
        out = [None] * self.size if self.rank == root else None
        dist.gather_object(obj, out, dst=root)
        return out

    def allgather(self, obj: Any) -> List[Any]:
        if self.size == 1:
            return [obj]
        out = [None] * self.size
        dist.all_gather_object(out, obj)
        return out

    def bcast(self, obj: Any, root: int = 0) -> Any:
        if self.size == 1:
            return obj
        box = [obj if self.rank == root else None]
        dist.broadcast_object_list(box, src=root)
        return box[0]

    def Barrier(self) -> None:
        if self.size > 1:
            dist.barrier()

    def Abort(self, code: int = 1) -> None:
        """Tear the job down (reference C:203-205).  The xGMI data plane is told first (the
        host abort word ends this rank's spinning kernels, every rank's failure word ends the
        peers' waits: ``fedmi.parallel.peer.abort_all``), then the RCCL communicator is aborted,
        which unblocks peers stuck in a collective; the launcher then kills the rest."""
        try:
            if "fedmi.parallel.peer" in sys.modules:
                sys.modules["fedmi.parallel.peer"].abort_all()
            if self.native is not None:
                self.native.abort()
        finally:
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(code)

    # ---- data plane ----
    def allreduce_(self, t: torch.Tensor, scale: Optional[float] = None) -> torch.Tensor:
        """In-place SUM over ranks on the current stream (fp32 / bf16 / fp64); with ``scale``,
        the sum of ``scale * t``.  (RCCL's pre-multiplied-sum op would fold the scale into the
        collective, but on this image's RCCL a one-rank communicator left the tail elements of
        some counts unscaled, e.g. 40001-40008 elements: past index 40000 -- so the scale is an
        explicit pass, or fused into the producer as in WideClient's bf16 buckets.)"""
        if self.size == 1:
            return t.mul_(scale) if scale is not None else t
        if t.is_cuda:
            if self.native is None and self.rccl_allowed:
                self.rccl()  # collective: every rank reaches this all-reduce together
            if self.native is not None:
                stream = torch.cuda.current_stream(t.device).cuda_stream
                if scale is not None:
                    t.mul_(scale)
                if t.dtype == torch.float32:
                    self.native.allreduce_f32(t.data_ptr(), t.numel(), stream)
                elif t.dtype == torch.bfloat16:
                    self.native.allreduce_bf16(t.data_ptr(), t.numel(), stream)
                elif t.dtype == torch.float64:
                    self.native.allreduce_f64(t.data_ptr(), t.numel(), stream)
                else:
                    raise TypeError(f"allreduce_: unsupported dtype {t.dtype}")
                return t
            if scale is not None:
                t.mul_(scale)
            if self._nccl_group is not None:
                dist.all_reduce(t, group=self._nccl_group)
            else:  # no device communicator: the host plane (gloo)
                t.copy_(self._host_sum_rank_order(t))
        else:
            if scale is not None:
                t.mul_(scale)
            dist.all_reduce(t)
        return t

    def _host_sum_rank_order(self, t: torch.Tensor) -> torch.Tensor:
        """Host plane of device all-reduces: every rank's buffer is all-gathered over gloo and
        summed as a left fold in rank order -- the order of the xGMI peer kernels, so a job that
        fell back to the host computes bit-identical FedAvg rounds (gloo's own reduction order
        depends on the world size)."""
        h = t.detach().cpu()
        parts = [torch.empty_like(h) for _ in range(self.size)]
        dist.all_gather(parts, h)
        acc = parts[0].clone()
        for p in parts[1:]:
            acc += p
        return acc

    def rccl_or_host(self):
        """COLLECTIVE.  The RCCL communicator (:meth:`rccl`), or ``None`` when RCCL is not
        allowed or its bootstrap failed -- then RCCL is disabled for the rest of the job and
        device all-reduces take the host plane.  Used by the round engine when the xGMI peer
        set-up fell back: every rank ends on the SAME next plane (the bootstrap's outcome is
        agreed, :meth:`rccl`), and a multi-GPU run still produces a (labelled) result."""
        try:
            return self.rccl()
        except (RuntimeError, TimeoutError) as e:
            self.rccl_allowed = False
            self.rccl_error = str(e)
            print(f"[fedmi] rank {self.rank}: RCCL unavailable ({e}); device all-reduces go through the host "
                  "(gloo, rank-order sums) -- data plane 'host'", file=sys.stderr, flush=True)
            return None

    def close(self) -> None:
        if self.native is not None:
            self.native.destroy()
            self.native = None
        if self._initialized_here and dist.is_initialized():
            dist.destroy_process_group()
            self._initialized_here = False


_WORLD: Optional[Comm] = None


def get_world(backend: str = "auto", device: Optional[str] = None, rccl: bool = True,
              rccl_proto: str = "LL") -> Comm:
    """Process-wide communicator (the analogue of ``MPI.COMM_WORLD``)."""
    global _WORLD
    if _WORLD is None:
        _WORLD = Comm(backend=backend, device=device, rccl=rccl, rccl_proto=rccl_proto)
    return _WORLD


def reset_world() -> None:
    global _WORLD
    if _WORLD is not None:
        _WORLD.close()
    _WORLD = None
