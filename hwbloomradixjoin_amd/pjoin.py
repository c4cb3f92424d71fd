"""The multi-GPU joins over torch.distributed: one process per GPU. The partitioned join
(include/hwbrj.h) runs either over the library's own RCCL communicator (comm_init +
join_partitioned_rccl: collectives on the join stream) or over torch.distributed callbacks
(TorchExchange: RCCL ("nccl") or gloo through host memory, for rehearsals with several ranks on one
GPU). set_filter_broadcast switches the replicated design to the north_star's bitmap broadcast.

SURVEY.md s8f row 3. Rank r of G owns radix partitions [r F / G, (r + 1) F / G): R chunks and
S survivors travel to the owner (variable all-to-alls), the owners' filter slices are all-gathered
(the filter broadcast, in 1/G pieces). The library runs every kernel and asks this module for the
exchanges through the hwbrj_exchange_t callbacks; device buffers are torch tensors (one per slot).
"""
from __future__ import annotations

import collections
import ctypes

import numpy as np

from . import _Stats, Stats, _BloomArgs, _err, _ptr, _check_rel, lib

_U64P = ctypes.POINTER(ctypes.c_uint64)
_BUFFER = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64)
_A2A_U64 = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, _U64P, _U64P, ctypes.c_uint64)
_A2AV = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, _U64P, _U64P, ctypes.c_int, _U64P, _U64P)
_AG = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64)


class _Exchange(ctypes.Structure):  # include/hwbrj.h hwbrj_exchange_t
    _fields_ = [("ctx", ctypes.c_void_p), ("buffer", _BUFFER), ("alltoall_u64", _A2A_U64),
                ("alltoallv", _A2AV), ("allgather", _AG)]


class TorchExchange:
    """hwbrj_exchange_t over torch.distributed. `group` None: the default group; with world 1 (or
    no process group) every exchange is a local copy. gloo groups stage through host memory."""

    NSLOTS = 9

    def __init__(self, device, group=None, force_collectives: bool = False):
        """force_collectives: run the process group's collectives even at world 1 (where every
        exchange is otherwise a local copy), so a one-GPU run exercises the RCCL branches."""
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.group = torch, dist, group
        self.device = torch.device(device)
        self.on = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if self.on else 1
        self.rank = dist.get_rank(group) if self.on else 0
        self.gloo = self.on and dist.get_backend(group) == "gloo"
        self.local = self.world == 1 and not (force_collectives and self.on)
        self.slots = [None] * self.NSLOTS
        self.error = None
        self.cuda = self.device.type == "cuda"
        self._c = _Exchange(None, _BUFFER(self._buffer), _A2A_U64(self._a2a_u64),
                            _A2AV(self._a2av), _AG(self._allgather))

    def _sync(self):
        if self.cuda:
            self.torch.cuda.synchronize(self.device)

    # every callback returns 0 / a pointer, or records the exception and fails (the library then
    # returns an error code and join_partitioned raises it)
    def _guard(self, fn, fail):
        try:
            return fn()
        except Exception as e:  # noqa: BLE001 (re-raised by join_partitioned)
            self.error = e
            return fail

    def _buffer(self, _ctx, slot, nbytes):
        def go():
            t = self.slots[slot]
            if t is None or t.numel() < nbytes:
                t = self.slots[slot] = self.torch.empty(max(int(nbytes), 16), dtype=self.torch.uint8,
                                                        device=self.device)
            return t.data_ptr()
        return self._guard(go, None)

    def _a2a_u64(self, _ctx, send, recv, n):
        def go():
            W = self.world
            s = np.ctypeslib.as_array(send, shape=(W * n,)).astype(np.int64)
            if self.local:
                np.ctypeslib.as_array(recv, shape=(n,))[:] = s
                return 0
            st = self.torch.from_numpy(s)
            if not self.gloo:
                st = st.to(self.device)
            rt = self.torch.empty_like(st)
            self.dist.all_to_all_single(rt, st, group=self.group)
            np.ctypeslib.as_array(recv, shape=(W * n,))[:] = rt.cpu().numpy().astype(np.uint64)
            return 0
        return self._guard(go, 1)

    def _a2av(self, _ctx, sslot, soff, sbytes, rslot, roff, rbytes):
        def go():
            W = self.world
            so, sb = [soff[j] for j in range(W)], [sbytes[j] for j in range(W)]
            ro, rb = [roff[j] for j in range(W)], [rbytes[j] for j in range(W)]
            # the library lays the blocks out consecutively (one all_to_all_single); it agrees on
            # every rank's status before each exchange, so no rank may bail out here alone
            src = self.slots[sslot][so[0]: so[-1] + sb[-1]]
            dst = self.slots[rslot][ro[0]: ro[-1] + rb[-1]]
            if self.local:
                dst.copy_(src)
                self._sync()  # (the library reads it on its own stream)
                return 0
            if self.gloo:
                out = self.torch.empty(dst.numel(), dtype=self.torch.uint8)
                self.dist.all_to_all_single(out, src.cpu(), rb, sb, group=self.group)
                dst.copy_(out)
            else:
                self.dist.all_to_all_single(dst, src, rb, sb, group=self.group)
            self._sync()
            return 0
        return self._guard(go, 1)

    def _allgather(self, _ctx, slot, nbytes):
        def go():
            W, r = self.world, self.rank
            full = self.slots[slot][: W * nbytes]
            if self.local:
                return 0
            mine = full[r * nbytes: (r + 1) * nbytes]
            if self.gloo:
                out = self.torch.empty(W * nbytes, dtype=self.torch.uint8)
                self.dist.all_gather_into_tensor(out, mine.cpu().clone(), group=self.group)
                full.copy_(out)
            else:
                self.dist.all_gather_into_tensor(full, mine.clone(), group=self.group)
            self._sync()
            return 0
        return self._guard(go, 1)


def join_partitioned(R, S, nR_total: int, args=None, exchange: TorchExchange | None = None) -> Stats:
    """This rank's part of the partitioned join of R and S (device (N, 2) int32 shards; nR_total =
    |R| over all ranks). Stats.filtered: this rank's S survivors; Stats.matches: the matches of its
    partitions -- both sum over ranks to the join's counts. ms_* fields are host wall times of the
    stages (ms_r_index: R exchange, ms_surv: slice all-gather + survivor exchange)."""
    _check_rel(R, S)
    x = exchange or TorchExchange(R.device)
    a = args._c() if args is not None else None
    st = _Stats()
    L = lib()
    rc = L.hwbrj_join_partitioned(ctypes.byref(x._c), x.rank, x.world, _ptr(R), R.shape[0],
                                  int(nR_total), _ptr(S), S.shape[0],
                                  ctypes.byref(a) if a is not None else None, ctypes.byref(st))
    if x.error is not None:
        e, x.error = x.error, None
        raise RuntimeError(f"hwbrj_join_partitioned: exchange failed: {e!r}") from e
    _err(rc, "hwbrj_join_partitioned")
    return Stats(**{n: getattr(st, n) for n, _ in _Stats._fields_})


def comm_init(group=None) -> tuple[int, int]:
    """The library's own RCCL communicator on the current device (hwbrj_comm_init): rank 0 of the
    torch.distributed group draws the unique id (hwbrj_comm_unique_id), the group broadcasts it,
    every rank joins. Without a process group: a world-1 communicator. Returns (world, rank)."""
    import torch
    import torch.distributed as dist
    L = lib()
    on = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size(group) if on else 1
    rank = dist.get_rank(group) if on else 0
    uid = (ctypes.c_uint8 * 128)()
    if rank == 0:
        _err(L.hwbrj_comm_unique_id(uid), "hwbrj_comm_unique_id")
    if on:
        t = torch.tensor(list(bytes(uid)), dtype=torch.uint8)
        if dist.get_backend(group) != "gloo":
            t = t.cuda()
        dist.broadcast(t, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        uid = (ctypes.c_uint8 * 128)(*t.cpu().tolist())
    _err(L.hwbrj_comm_init(uid, world, rank), "hwbrj_comm_init")
    return world, rank


def comm_destroy() -> None:
    _err(lib().hwbrj_comm_destroy(), "hwbrj_comm_destroy")


def set_filter_broadcast(on: bool) -> None:
    """The replicated design with the north_star's bitmap broadcast (hwbrj_set_filter_broadcast):
    rank 0 builds the filter slices, ncclBroadcast delivers them to every rank. Needs comm_init."""
    _err(lib().hwbrj_set_filter_broadcast(1 if on else 0), "hwbrj_set_filter_broadcast")


def join_partitioned_rccl(R, S, nR_total: int, args=None) -> Stats:
    """join_partitioned over the library's own RCCL communicator (comm_init first): the all-to-alls
    and the slice all-gather are RCCL calls on the join stream, no Python in between."""
    _check_rel(R, S)
    a = args._c() if args is not None else None
    st = _Stats()
    rc = lib().hwbrj_join_partitioned_rccl(_ptr(R), R.shape[0], int(nR_total), _ptr(S), S.shape[0],
                                           ctypes.byref(a) if a is not None else None, ctypes.byref(st))
    _err(rc, "hwbrj_join_partitioned_rccl")
    return Stats(**{n: getattr(st, n) for n, _ in _Stats._fields_})


# What every enqueued async partitioned join reads until its wait returns: its R and S tensors and,
# over the callbacks, the TorchExchange (its ctypes thunks and the device buffers of its exchanges;
# a wait that reruns the join calls the thunks again). Held here, in call order, and released by
# join_partitioned_wait, so a caller that drops its own references cannot free them early.
_inflight = collections.deque()


def join_partitioned_rccl_async(R, S, nR_total: int, args=None) -> None:
    """join_partitioned_rccl enqueued without host waits (hwbrj_join_partitioned_rccl_async): the
    exchanges are padded to a plan made by an earlier synchronous join of the same shapes (the first
    call runs synchronously and makes it). Collect with join_partitioned_wait, in call order; R and
    S must stay unchanged until then (this module keeps them alive). A collective: every rank makes
    the same calls."""
    _check_rel(R, S)
    a = args._c() if args is not None else None
    rc = lib().hwbrj_join_partitioned_rccl_async(_ptr(R), R.shape[0], int(nR_total), _ptr(S), S.shape[0],
                                                 ctypes.byref(a) if a is not None else None)
    _err(rc, "hwbrj_join_partitioned_rccl_async")
    _inflight.append((R, S, None))


def join_partitioned_async(R, S, nR_total: int, args, exchange: "TorchExchange") -> None:
    """The async partitioned join over torch.distributed callbacks (hwbrj_join_partitioned_async):
    the same plan and padded layout as join_partitioned_rccl_async, with host-synchronous exchanges
    (ranks may share a GPU: gloo). Collect with join_partitioned_wait. `exchange` is required (one
    TorchExchange per rank, reused across joins); it, R and S are kept alive until the wait."""
    if not isinstance(exchange, TorchExchange):
        raise TypeError("join_partitioned_async needs the rank's TorchExchange (exchange=...)")
    _check_rel(R, S)
    x = exchange
    a = args._c() if args is not None else None
    rc = lib().hwbrj_join_partitioned_async(ctypes.byref(x._c), x.rank, x.world, _ptr(R), R.shape[0],
                                            int(nR_total), _ptr(S), S.shape[0],
                                            ctypes.byref(a) if a is not None else None)
    if x.error is not None:
        e, x.error = x.error, None
        raise RuntimeError(f"hwbrj_join_partitioned_async: exchange failed: {e!r}") from e
    _err(rc, "hwbrj_join_partitioned_async")
    _inflight.append((R, S, x))


def join_partitioned_wait() -> Stats:
    """The oldest enqueued async partitioned join's result (hwbrj_join_partitioned_wait); a join
    whose padded blocks overflowed on any rank is rerun synchronously here (same counts)."""
    st = _Stats()
    try:
        _err(lib().hwbrj_join_partitioned_wait(ctypes.byref(st)), "hwbrj_join_partitioned_wait")
    finally:
        if _inflight:
            _inflight.popleft()
    return Stats(**{n: getattr(st, n) for n, _ in _Stats._fields_})


PJ_INFO_FIELDS = ("plan_valid", "BR", "BI", "BW", "async_joins", "sync_plan_joins", "overflow_reruns",
                  "plans", "in_flight", "last_rerun_flag", "last_r_block", "last_item_block",
                  "last_word_block")


def pj_async_info() -> dict:
    """hwbrj_pj_async_info: the async join's plan (block bounds) and counters."""
    out = (ctypes.c_uint64 * 16)()
    _err(lib().hwbrj_pj_async_info(out), "hwbrj_pj_async_info")
    return {k: int(out[i]) for i, k in enumerate(PJ_INFO_FIELDS)}


def _bind(L):
    L.hwbrj_join_partitioned_rccl_async.restype = ctypes.c_int
    L.hwbrj_join_partitioned_rccl_async.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                                    ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(_BloomArgs)]
    L.hwbrj_join_partitioned_async.restype = ctypes.c_int
    L.hwbrj_join_partitioned_async.argtypes = [ctypes.POINTER(_Exchange), ctypes.c_int, ctypes.c_int,
                                               ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                               ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(_BloomArgs)]
    L.hwbrj_join_partitioned_wait.restype = ctypes.c_int
    L.hwbrj_join_partitioned_wait.argtypes = [ctypes.POINTER(_Stats)]
    L.hwbrj_pj_async_info.restype = ctypes.c_int
    L.hwbrj_pj_async_info.argtypes = [ctypes.c_void_p]
    L.hwbrj_comm_unique_id.restype = ctypes.c_int
    L.hwbrj_comm_unique_id.argtypes = [ctypes.c_void_p]
    L.hwbrj_comm_init.restype = ctypes.c_int
    L.hwbrj_comm_init.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    L.hwbrj_comm_destroy.restype = ctypes.c_int
    L.hwbrj_set_filter_broadcast.restype = ctypes.c_int
    L.hwbrj_set_filter_broadcast.argtypes = [ctypes.c_int]
    L.hwbrj_join_partitioned_rccl.restype = ctypes.c_int
    L.hwbrj_join_partitioned_rccl.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                              ctypes.c_void_p, ctypes.c_uint64,
                                              ctypes.POINTER(_BloomArgs), ctypes.POINTER(_Stats)]
    L.hwbrj_join_partitioned.restype = ctypes.c_int
    L.hwbrj_join_partitioned.argtypes = [ctypes.POINTER(_Exchange), ctypes.c_int, ctypes.c_int,
                                         ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                         ctypes.c_void_p, ctypes.c_uint64,
                                         ctypes.POINTER(_BloomArgs), ctypes.POINTER(_Stats)]


_bind(lib())
