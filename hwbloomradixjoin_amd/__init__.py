"""hwbloomradixjoin_amd -- MI355X-native bloom-filtered radix hash join.

Python mirror of the reference's operator interface for the BPRO path
(Briimbo/HwBloomRadixJoin src/parallel_radix_join_bloom.h:34-36, src/parallel_radix_join.h:33-34,
src/bloom_filter.h:10,50-55, src/types.h:37-63), bound over ctypes to the C-ABI library
``libhwbrj.so`` (include/hwbrj.h). The join runs only in the HIP kernels of that library: if the
library is missing this package raises instead of falling back to anything on the CPU.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

__all__ = [
    "BASIC", "BLOCKED", "SECTORIZED", "BloomFilterArgs", "Relation", "Result", "Stats",
    "BPRO", "PRO", "join_materialize_device", "set_materialize", "set_gpus", "BPRH", "BPRHO", "BRJ", "PRH", "PRHO", "RJ", "assert_args", "join_device", "join_device_async", "join_wait", "join_wait_all", "set_async_timing", "generate_device", "generate_device_range",
    "generate_host", "nonunique_threshold", "create_relation_nonunique",
    "create_relation_nonunique_from_pk", "create_relation_fk_from_pk", "create_relation_zipf",
    "rand_stream", "reference_relations", "create_relation_zipf_device",
    "export_filter", "hash_crc", "hash_crapwow", "lib", "LIB_PATH", "shard_range", "write_relation",
]

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HWBRJ_LIB") or os.path.join(PKG_DIR, "libhwbrj.so")  # HWBRJ_LIB: dev-only variant builds
CLI_PATH = os.path.join(PKG_DIR, "mchashjoins")

# src/bloom_filter.h:10 (BASIC, BLOCKED) + this build's SECTORIZED
BASIC, BLOCKED, SECTORIZED = 0, 1, 2
_VARIANTS = {"basic": BASIC, "blocked": BLOCKED, "sectorized": SECTORIZED}


class _Tuple(ctypes.Structure):  # src/types.h:37-40
    _fields_ = [("key", ctypes.c_int32), ("payload", ctypes.c_int32)]


class _Relation(ctypes.Structure):  # src/types.h:46-49
    _fields_ = [("tuples", ctypes.POINTER(_Tuple)), ("num_tuples", ctypes.c_uint64)]


class _Result(ctypes.Structure):  # src/types.h:59-63
    _fields_ = [("totalresults", ctypes.c_int64), ("resultlist", ctypes.c_void_p),
                ("nthreads", ctypes.c_int)]


class _BloomArgs(ctypes.Structure):  # src/bloom_filter.h:50-55
    _fields_ = [("variant", ctypes.c_int), ("m", ctypes.c_uint64), ("k", ctypes.c_uint64),
                ("B", ctypes.c_uint64)]


class _Stats(ctypes.Structure):  # include/hwbrj.h hwbrj_stats_t
    _fields_ = [("filtered", ctypes.c_uint64), ("matches", ctypes.c_int64), ("mode", ctypes.c_int),
                ("format", ctypes.c_int), ("partitions", ctypes.c_uint32),
                ("subparts", ctypes.c_uint32), ("slice_segments", ctypes.c_uint32)] + [
                    (n, ctypes.c_double) for n in (
                        "ms_total", "ms_r_scatter", "ms_r_index", "ms_build", "ms_s_scatter",
                        "ms_s_index", "ms_probe", "ms_surv", "ms_join", "ms_join_probe")] + [
                    ("join_keys", ctypes.c_int), ("unstaged_items", ctypes.c_uint32),
                    ("join_key_bits", ctypes.c_uint32)]

# hwbrj_stats_t.join_keys (include/hwbrj.h): the key format between the build / probe and the join
JOIN_KEYS_32, JOIN_KEYS_PACKED, JOIN_KEYS_MIXED = 0, 1, 2


_LIB = None


def lib() -> ctypes.CDLL:
    """Load libhwbrj.so (built by __graft_entry__.build()). Raises if it is missing."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; "
                              "g.build()'` (the MI355X HIP library is required; there is no CPU "
                              "fallback)")
        # torch-ROCm ships its own HIP runtime. If libhwbrj.so (linked against /opt/rocm's) is
        # loaded first, torch's later device init leaves this library's runtime with no devices
        # ("no ROCm-capable device"); loading torch's libraries first makes the two coexist.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        L.BPRO.restype = ctypes.POINTER(_Result)
        L.BPRO.argtypes = [ctypes.POINTER(_Relation), ctypes.POINTER(_Relation), ctypes.c_int,
                           ctypes.POINTER(_BloomArgs)]
        L.PRO.restype = ctypes.POINTER(_Result)
        L.PRO.argtypes = [ctypes.POINTER(_Relation), ctypes.POINTER(_Relation), ctypes.c_int]
        for nm in ("BPRH", "BPRHO", "BRJ"):
            getattr(L, nm).restype = ctypes.POINTER(_Result)
            getattr(L, nm).argtypes = L.BPRO.argtypes
        for nm in ("PRH", "PRHO", "RJ"):
            getattr(L, nm).restype = ctypes.POINTER(_Result)
            getattr(L, nm).argtypes = L.PRO.argtypes
        L.assert_args.argtypes = [ctypes.POINTER(_BloomArgs)]
        L.hwbrj_join_device.restype = ctypes.c_int
        L.hwbrj_join_device_async.restype = ctypes.c_int
        L.hwbrj_join_device_async.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                              ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
        L.hwbrj_join_device_algo.restype = ctypes.c_int
        L.hwbrj_join_device_algo.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                             ctypes.c_uint64, ctypes.POINTER(_BloomArgs),
                                             ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(_Stats)]
        L.hwbrj_join_wait.restype = ctypes.c_int
        L.hwbrj_join_wait.argtypes = [ctypes.c_void_p]
        L.hwbrj_set_async_timing.restype = ctypes.c_int
        L.hwbrj_set_async_timing.argtypes = [ctypes.c_int]
        L.hwbrj_join_wait_all.restype = ctypes.c_int
        L.hwbrj_join_wait_all.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        L.hwbrj_join_device.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                        ctypes.c_uint64, ctypes.POINTER(_BloomArgs),
                                        ctypes.c_void_p, ctypes.POINTER(_Stats)]
        L.hwbrj_join_materialize_device.restype = ctypes.c_int
        L.hwbrj_join_materialize_device.argtypes = [
            ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
            ctypes.POINTER(_BloomArgs), ctypes.c_void_p, ctypes.c_uint64,
            ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p, ctypes.POINTER(_Stats),
            ctypes.POINTER(ctypes.c_double)]
        L.hwbrj_set_materialize.restype = None
        L.hwbrj_set_materialize.argtypes = [ctypes.c_int]
        L.hwbrj_set_gpus.restype = ctypes.c_int
        L.hwbrj_set_gpus.argtypes = [ctypes.c_int]
        L.hwbrj_generate_device.restype = ctypes.c_int
        L.hwbrj_generate_device.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                            ctypes.c_uint64, ctypes.c_uint64, ctypes.c_double,
                                            ctypes.c_uint64, ctypes.c_void_p]
        L.hwbrj_generate_device_range.restype = ctypes.c_int
        L.hwbrj_generate_device_range.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                                  ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                                  ctypes.c_uint64, ctypes.c_double, ctypes.c_uint64,
                                                  ctypes.c_void_p]
        L.hwbrj_generate_host.restype = ctypes.c_int
        L.hwbrj_generate_host.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                          ctypes.c_uint64, ctypes.c_uint64, ctypes.c_double,
                                          ctypes.c_uint64, ctypes.c_int]
        L.hwbrj_nonunique_threshold.restype = ctypes.c_uint64
        L.hwbrj_nonunique_threshold.argtypes = [ctypes.c_uint64, ctypes.c_double, ctypes.c_int]
        L.hwbrj_create_relation_nonunique.restype = ctypes.c_int
        L.hwbrj_create_relation_nonunique.argtypes = [ctypes.c_void_p, ctypes.c_uint64,
                                                      ctypes.c_int64, ctypes.c_uint32]
        for fn in (L.hwbrj_create_relation_nonunique_from_pk, L.hwbrj_create_relation_fk_from_pk):
            fn.restype = ctypes.c_int
            fn.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                           ctypes.c_int64, ctypes.c_double, ctypes.c_uint32]
        L.hwbrj_create_relation_zipf.restype = ctypes.c_int
        L.hwbrj_create_relation_zipf.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                                 ctypes.c_double, ctypes.c_uint32, ctypes.c_int]
        L.hwbrj_create_relation_zipf_device.restype = ctypes.c_int
        L.hwbrj_create_relation_zipf_device.argtypes = [
            ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_double, ctypes.c_uint32,
            ctypes.c_double, ctypes.c_int, ctypes.c_void_p]
        L.hwbrj_rand_stream.restype = ctypes.c_int
        L.hwbrj_rand_stream.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64]
        L.hwbrj_write_relation.restype = ctypes.c_int
        L.hwbrj_write_relation.argtypes = [ctypes.POINTER(_Relation), ctypes.c_char_p]
        L.hwbrj_write_result_relation.restype = ctypes.c_int
        L.hwbrj_write_result_relation.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
        L.hwbrj_export_filter.restype = ctypes.c_int
        L.hwbrj_export_filter.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        L.hwbrj_hash_crc.restype = ctypes.c_uint32
        L.hwbrj_hash_crc.argtypes = [ctypes.c_uint32, ctypes.c_int32]
        L.hwbrj_hash_crapwow.restype = ctypes.c_uint32
        L.hwbrj_hash_crapwow.argtypes = [ctypes.c_uint32, ctypes.c_int32]
        L.hwbrj_device_count.restype = ctypes.c_int
        L.hwbrj_set_device.restype = ctypes.c_int
        L.hwbrj_set_device.argtypes = [ctypes.c_int]
        L.hwbrj_last_error.restype = ctypes.c_char_p
        L.hwbrj_version.restype = ctypes.c_char_p
        L.hwbrj_set_test_hook.restype = ctypes.c_int
        L.hwbrj_set_test_hook.argtypes = [ctypes.c_int, ctypes.c_int64]
        L.hwbrj_tsc_hz.restype = ctypes.c_uint64
        L.hwbrj_copy_bandwidth.restype = ctypes.c_int
        L.hwbrj_copy_bandwidth.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
        L.hwbrj_release.restype = None
        _LIB = L
    return _LIB


def _err(code: int, what: str):
    if code != 0:
        raise RuntimeError(f"{what} failed ({code}): {lib().hwbrj_last_error().decode()}")


@dataclass
class BloomFilterArgs:
    """src/bloom_filter.h:50-55. Defaults are src/main.c:389-393 (variant BASIC, m=256 Mi, k=8,
    B=1024)."""
    variant: int = BASIC
    m: int = 256 << 20
    k: int = 8
    B: int = 1024

    @classmethod
    def from_flag(cls, b: str, m: int, k: int, B: int = 1024) -> Optional["BloomFilterArgs"]:
        """The CLI's -b parsing (src/main.c:692-698): 'no' -> None; unknown -> BASIC, except
        'sectorized' which selects this build's SECTORIZED variant."""
        if b == "no":
            return None
        return cls(_VARIANTS.get(b, BASIC), m, k, B)

    def _c(self) -> _BloomArgs:
        return _BloomArgs(int(self.variant), int(self.m), int(self.k), int(self.B))


@dataclass
class Result:
    """src/types.h:59-63. `pairs` holds the materialized {R.payload, S.payload} result
    (JOIN_RESULT_MATERIALIZE, see set_materialize), else None (the reference's default build)."""
    totalresults: int
    nthreads: int
    pairs: Optional[np.ndarray] = None


class _TupleBuffer(ctypes.Structure):  # src/tuple_buffer.h:27-30
    pass


_TupleBuffer._fields_ = [("tuples", ctypes.POINTER(_Tuple)), ("next", ctypes.POINTER(_TupleBuffer))]


class _ChainedTupleBuffer(ctypes.Structure):  # src/tuple_buffer.h:32-40
    _fields_ = [("buf", ctypes.POINTER(_TupleBuffer)), ("readcursor", ctypes.POINTER(_TupleBuffer)),
                ("writecursor", ctypes.POINTER(_TupleBuffer)), ("writepos", ctypes.c_uint32),
                ("readpos", ctypes.c_uint32), ("readlen", ctypes.c_uint32),
                ("numbufs", ctypes.c_uint32)]


class _ThreadResult(ctypes.Structure):  # src/types.h:51-56
    _fields_ = [("nresults", ctypes.c_int64), ("results", ctypes.c_void_p),
                ("threadid", ctypes.c_uint32)]


_CB_TUPLES = 1024 * 1024  # CHAINEDBUFF_NUMTUPLESPERBUF


def _take_result(r) -> Result:
    """Copy a result_t (and its chained result buffers, if materialized) and free it."""
    libc = ctypes.CDLL(None)
    res = r.contents
    pairs = None
    if res.resultlist:
        tl = ctypes.cast(res.resultlist, ctypes.POINTER(_ThreadResult))
        parts = []
        for t in range(res.nthreads):
            cb = ctypes.cast(tl[t].results, ctypes.POINTER(_ChainedTupleBuffer)).contents
            n, b, first = tl[t].nresults, cb.buf, True
            while b and n > 0:  # cb_begin / cb_read_next order: newest buffer first
                take = min(n, cb.writepos if first else _CB_TUPLES)
                a = np.ctypeslib.as_array(ctypes.cast(b.contents.tuples, ctypes.POINTER(ctypes.c_int32)),
                                          shape=(take * 2,))
                parts.append(a.reshape(-1, 2).copy())
                n -= take
                b, first = b.contents.next, False
            addr = ctypes.cast(cb.buf, ctypes.c_void_p).value
            while addr:  # (plain addresses: a ctypes field view would read freed memory)
                b = ctypes.cast(addr, ctypes.POINTER(_TupleBuffer)).contents
                nxt = ctypes.cast(b.next, ctypes.c_void_p).value
                libc.free(ctypes.cast(b.tuples, ctypes.c_void_p))
                libc.free(ctypes.c_void_p(addr))
                addr = nxt
            libc.free(ctypes.c_void_p(tl[t].results))
        libc.free(ctypes.cast(res.resultlist, ctypes.c_void_p))
        pairs = np.concatenate(parts) if parts else np.empty((0, 2), dtype=np.int32)
    out = Result(res.totalresults, res.nthreads, pairs)
    libc.free(r)
    return out


# include/hwbrj.h hwbrj_set_test_hook
HOOK_JOIN_SPLIT, HOOK_PJ_FAIL_RANK, HOOK_BCAST_NONROOT, HOOK_PJ_PLAN_DIV, HOOK_PJ_ASYNC_FAIL = 1, 2, 3, 4, 5
_HOOK_OFF = {HOOK_JOIN_SPLIT: 0, HOOK_PJ_FAIL_RANK: -1, HOOK_BCAST_NONROOT: 0, HOOK_PJ_PLAN_DIV: 0,
             HOOK_PJ_ASYNC_FAIL: 0}


def version() -> str:
    """hwbrj_version(): name, version and every non-default compile-time knob ("knobs: ...")."""
    return lib().hwbrj_version().decode()


def set_test_hook(hook: int, value: int) -> None:
    """hwbrj_set_test_hook: force a rarely taken path or inject a failure (tests only)."""
    _err(lib().hwbrj_set_test_hook(hook, int(value)), "hwbrj_set_test_hook")


@contextlib.contextmanager
def hooked(hook: int, value: int):
    """set_test_hook for the duration of a with-block (then off again)."""
    set_test_hook(hook, value)
    try:
        yield
    finally:
        set_test_hook(hook, _HOOK_OFF[hook])


def set_gpus(gpus: int) -> None:
    """Shards of S for host BPRO/PRO (hwbrj_set_gpus): shard g on visible device g mod
    device_count, R replicated, counts summed. 0 restores the default (HWBRJ_GPUS, else 1)."""
    _err(lib().hwbrj_set_gpus(int(gpus)), "hwbrj_set_gpus")


def set_materialize(on: bool) -> None:
    """Materialize {R.payload, S.payload} pairs in BPRO/PRO results (JOIN_RESULT_MATERIALIZE)."""
    lib().hwbrj_set_materialize(1 if on else 0)


@dataclass
class Stats:
    filtered: int
    matches: int
    mode: int
    format: int
    partitions: int
    subparts: int
    slice_segments: int
    ms_total: float
    ms_r_scatter: float
    ms_r_index: float
    ms_build: float
    ms_s_scatter: float
    ms_s_index: float
    ms_probe: float
    ms_surv: float
    ms_join: float
    ms_join_probe: float
    join_keys: int = 0       # JOIN_KEYS_32 / _PACKED / _MIXED
    unstaged_items: int = 0  # probe items whose survivors overflowed the LDS stage
    join_key_bits: int = 32  # bits per packed join key (18 at the north star, 24, or 32: codes)


class Relation:
    """relation_t over a contiguous (N, 2) int32 array of {key, payload} (src/types.h:37-49)."""

    def __init__(self, tuples: np.ndarray):
        t = np.ascontiguousarray(tuples, dtype=np.int32)
        if t.ndim != 2 or t.shape[1] != 2:
            raise ValueError("tuples must have shape (N, 2): key, payload")
        self.tuples = t
        self._c = _Relation(t.ctypes.data_as(ctypes.POINTER(_Tuple)), t.shape[0])

    @property
    def num_tuples(self) -> int:
        return self.tuples.shape[0]


def write_relation(rel: "Relation | np.ndarray", filename: str) -> None:
    """src/generator.c:250-263 write_relation (hwbrj_write_relation): a "#KEY, VAL" header, then
    "key payload" lines; the CLI's -R / -S read it back."""
    r = rel if isinstance(rel, Relation) else Relation(rel)
    _err(lib().hwbrj_write_relation(ctypes.byref(r._c), os.fsencode(filename)), "hwbrj_write_relation")


def assert_args(args: BloomFilterArgs) -> bool:
    """src/bloom_filter.c:25-34 without the exit(1): True when the reference would accept."""
    m, B = int(args.m), int(args.B)
    if m & (m - 1):
        return False
    if args.variant != BASIC and (B <= 0 or B & (B - 1) or m % B):
        return False
    return True


def BPRO(relR: Relation, relS: Relation, nthreads: int, args: BloomFilterArgs) -> Result:
    """src/parallel_radix_join_bloom.c:1781-1787 on the MI355X (prints the reference's lines)."""
    a = args._c()
    return _take_result(lib().BPRO(ctypes.byref(relR._c), ctypes.byref(relS._c), int(nthreads),
                                   ctypes.byref(a)))


def PRO(relR: Relation, relS: Relation, nthreads: int) -> Result:
    """src/parallel_radix_join.c:1697-1700 (no filter) on the MI355X."""
    return _take_result(lib().PRO(ctypes.byref(relR._c), ctypes.byref(relS._c), int(nthreads)))


def _run(name: str, relR: Relation, relS: Relation, nthreads: int, args=None) -> Result:
    fn = getattr(lib(), name)
    r = (fn(ctypes.byref(relR._c), ctypes.byref(relS._c), int(nthreads), ctypes.byref(args._c()))
         if args is not None else fn(ctypes.byref(relR._c), ctypes.byref(relS._c), int(nthreads)))
    return _take_result(r)


def BPRH(relR, relS, nthreads, args):
    """src/parallel_radix_join_bloom.c:1789-1795 (same MI355X operator as BPRO)."""
    return _run("BPRH", relR, relS, nthreads, args)


def BPRHO(relR, relS, nthreads, args):
    """src/parallel_radix_join_bloom.c:1797-1804 (same MI355X operator as BPRO)."""
    return _run("BPRHO", relR, relS, nthreads, args)


def BRJ(relR, relS, nthreads, args):
    """src/parallel_radix_join_bloom.c:1806-1930 (same MI355X operator as BPRO)."""
    return _run("BRJ", relR, relS, nthreads, args)


def PRH(relR, relS, nthreads):
    return _run("PRH", relR, relS, nthreads)


def PRHO(relR, relS, nthreads):
    return _run("PRHO", relR, relS, nthreads)


def RJ(relR, relS, nthreads):
    return _run("RJ", relR, relS, nthreads)


def _ptr(t) -> int:
    return int(t.data_ptr())


def _check_rel(R, S):
    """Both relations: contiguous (N, 2) torch.int32 tensors ({key, payload}) on one GPU. The
    library's current HIP device is switched to that GPU (the join runs on its Engine)."""
    import torch
    for name, t in (("R", R), ("S", S)):
        if (not t.is_cuda or t.dtype != torch.int32 or t.dim() != 2 or t.shape[1] != 2
                or not t.is_contiguous()):
            raise ValueError(f"{name} must be a contiguous (N, 2) torch.int32 tensor on the GPU")
    if R.device != S.device:
        raise ValueError(f"R is on {R.device} but S is on {S.device}")
    _err(lib().hwbrj_set_device(R.device.index or 0), "hwbrj_set_device")


def join_device_async(R, S, args: Optional[BloomFilterArgs] = None, stream=None) -> None:
    """Enqueue the join of device tensors R, S without waiting (hwbrj_join_device_async);
    join_wait() returns the Stats of the last join enqueued on this device (counts; an async join
    records no phase events, so its ms_* fields are 0)."""
    _check_rel(R, S)
    a = args._c() if args is not None else None
    sp = ctypes.c_void_p(stream.cuda_stream) if stream is not None else None
    _err(lib().hwbrj_join_device_async(_ptr(R), R.shape[0], _ptr(S), S.shape[0],
                                       ctypes.byref(a) if a is not None else None, sp),
         "hwbrj_join_device_async")


def join_wait() -> Stats:
    """Wait for the last enqueued join on this device and return its Stats."""
    st = _Stats()
    _err(lib().hwbrj_join_wait(ctypes.byref(st)), "hwbrj_join_wait")
    return Stats(**{n: getattr(st, n) for n, _ in _Stats._fields_})


def set_async_timing(on: bool) -> None:
    """hwbrj_set_async_timing: async joins time their S scatter on the side stream that runs it
    (Stats.ms_s_scatter of every async join); off by default."""
    _err(lib().hwbrj_set_async_timing(1 if on else 0), "hwbrj_set_async_timing")


def join_wait_all(capacity: int = 256) -> list:
    """Wait for the last enqueued join and return the Stats of EVERY join enqueued on this device
    since the last join_wait / join_wait_all, oldest first (hwbrj_join_wait_all: each join keeps its
    own counts in a device ring). Raises if more than `capacity` joins are pending."""
    arr = (_Stats * max(1, capacity))()
    n = ctypes.c_int(0)
    _err(lib().hwbrj_join_wait_all(arr, capacity, ctypes.byref(n)), "hwbrj_join_wait_all")
    return [Stats(**{f: getattr(arr[i], f) for f, _ in _Stats._fields_}) for i in range(n.value)]


ALGO_PRO, ALGO_PRH, ALGO_PRHO = 0, 1, 2  # include/hwbrj.h HWBRJ_ALGO_* (per-partition join)


def join_device(R, S, args: Optional[BloomFilterArgs] = None, stream=None,
                algorithm: int = ALGO_PRO) -> Stats:
    """Join device-resident torch int32 tensors of shape (N, 2) ({key, payload}) in HBM.
    args=None runs PRO. `stream` is a torch.cuda.Stream (default: the library's own stream).
    algorithm: the per-partition join (ALGO_PRO bucket chaining's role, ALGO_PRH / ALGO_PRHO the
    histogram joins of src/parallel_radix_join_bloom.c:350-555)."""
    _check_rel(R, S)
    st = _Stats()
    a = args._c() if args is not None else None
    sp = ctypes.c_void_p(stream.cuda_stream) if stream is not None else None
    rc = lib().hwbrj_join_device_algo(_ptr(R), R.shape[0], _ptr(S), S.shape[0],
                                      ctypes.byref(a) if a is not None else None, int(algorithm),
                                      sp, ctypes.byref(st))
    _err(rc, "hwbrj_join_device_algo")
    return Stats(**{n: getattr(st, n) for n, _ in _Stats._fields_})


def join_materialize_device(R, S, args: Optional[BloomFilterArgs] = None, stream=None,
                            capacity: Optional[int] = None):
    """(Stats, pairs, ms): the join of device tensors R, S with its result materialized as a (n, 2)
    int32 GPU tensor of {R.payload, S.payload} pairs, unordered (JOIN_RESULT_MATERIALIZE); ms is
    the device time of the materializing pipeline. capacity: output rows to allocate (None: sized
    by a counting join first; too small: the pipeline runs again at the exact size)."""
    import torch
    if capacity is None:
        capacity = join_device(R, S, args, stream).matches
    a = args._c() if args is not None else None
    sp = ctypes.c_void_p(stream.cuda_stream) if stream is not None else None
    for _ in range(2):
        out = torch.empty((max(int(capacity), 1), 2), dtype=torch.int32, device=R.device)
        n = ctypes.c_uint64()
        st2 = _Stats()
        ms = ctypes.c_double()
        rc = lib().hwbrj_join_materialize_device(_ptr(R), R.shape[0], _ptr(S), S.shape[0],
                                                 ctypes.byref(a) if a is not None else None,
                                                 _ptr(out), out.shape[0], ctypes.byref(n), sp,
                                                 ctypes.byref(st2), ctypes.byref(ms))
        if rc != 7:
            break
        capacity = n.value
    _err(rc, "hwbrj_join_materialize_device")
    stats = Stats(**{f: getattr(st2, f) for f, _ in _Stats._fields_})
    return stats, out[: n.value], ms.value


def copy_bandwidth(nbytes: int = 4 << 30, reps: int = 5) -> float:
    """GB/s of a streaming device copy ((read + write) bytes / median time; hwbrj_copy_bandwidth):
    the measured copy rate the roofline reports beside the 8 TB/s spec peak."""
    g = ctypes.c_double()
    _err(lib().hwbrj_copy_bandwidth(int(nbytes), int(reps), ctypes.byref(g)), "hwbrj_copy_bandwidth")
    return g.value


def generate_device(out, nthreads: int, maxid: int, threshold: int, selectivity: float,
                    seed: int, stream=None) -> None:
    """Fill a (N, 2) int32 GPU tensor with the reference generator's multiset
    (src/generator.c:304-415), seeded permuted order, payload = row index."""
    sp = ctypes.c_void_p(stream.cuda_stream) if stream is not None else None
    _err(lib().hwbrj_generate_device(_ptr(out), out.shape[0], nthreads, maxid, threshold,
                                     selectivity, seed, sp), "hwbrj_generate_device")


def generate_device_range(out, n: int, offset: int, nthreads: int, maxid: int, threshold: int,
                          selectivity: float, seed: int, stream=None) -> None:
    """Rows [offset, offset + out.shape[0]) of the n-row relation generate_device would build."""
    sp = ctypes.c_void_p(stream.cuda_stream) if stream is not None else None
    _err(lib().hwbrj_generate_device_range(_ptr(out), n, offset, out.shape[0], nthreads, maxid,
                                           threshold, selectivity, seed, sp),
         "hwbrj_generate_device_range")


def generate_host(n: int, nthreads: int, maxid: int, threshold: int, selectivity: float,
                  seed: int, host_threads: int = 0) -> np.ndarray:
    """The same relation as generate_device, on the host: (n, 2) int32."""
    out = np.empty((n, 2), dtype=np.int32)
    _err(lib().hwbrj_generate_host(out.ctypes.data, n, nthreads, maxid, threshold, selectivity,
                                   seed, host_threads), "hwbrj_generate_host")
    return out


def nonunique_threshold(r_size: int, selectivity: float, full_range: bool) -> int:
    """src/main.c:421-427: the key bound of --non-unique / --full-range relations."""
    return int(lib().hwbrj_nonunique_threshold(r_size, selectivity, 1 if full_range else 0))


def create_relation_nonunique(n: int, maxid: int, seed: int) -> np.ndarray:
    """src/generator.c:585-605 after srand(seed): n random keys in [0, maxid), payload = row."""
    out = np.empty((n, 2), dtype=np.int32)
    _err(lib().hwbrj_create_relation_nonunique(out.ctypes.data, n, maxid, seed),
         "hwbrj_create_relation_nonunique")
    return out


def _from_pk(fn, name, n, pk, threshold, selectivity, seed):
    pk = np.ascontiguousarray(pk, dtype=np.int32)
    out = np.empty((n, 2), dtype=np.int32)
    _err(fn(out.ctypes.data, n, pk.ctypes.data, pk.shape[0], threshold, selectivity, seed), name)
    return out


def create_relation_nonunique_from_pk(n: int, pk: np.ndarray, threshold: int, selectivity: float,
                                      seed: int) -> np.ndarray:
    """src/generator.c:608-646 (the --non-unique S relation)."""
    return _from_pk(lib().hwbrj_create_relation_nonunique_from_pk,
                    "hwbrj_create_relation_nonunique_from_pk", n, pk, threshold, selectivity, seed)


def create_relation_fk_from_pk(n: int, pk: np.ndarray, threshold: int, selectivity: float,
                               seed: int) -> np.ndarray:
    """src/generator.c:531-582 (the --full-range S relation)."""
    return _from_pk(lib().hwbrj_create_relation_fk_from_pk, "hwbrj_create_relation_fk_from_pk",
                    n, pk, threshold, selectivity, seed)


def create_relation_zipf(n: int, alphabet_size: int, theta: float, seed: int,
                         host_threads: int = 0) -> np.ndarray:
    """src/generator.c:659-676 + src/genzipf.c:28-158 (the -z S relation), payload = row."""
    out = np.empty((n, 2), dtype=np.int32)
    _err(lib().hwbrj_create_relation_zipf(out.ctypes.data, n, alphabet_size, theta, seed,
                                          host_threads), "hwbrj_create_relation_zipf")
    return out


def create_relation_zipf_device(out, alphabet_size: int, theta: float, seed: int,
                                selectivity: float = 1.0, host_threads: int = 0) -> None:
    """The -z relation into a (n, 2) int32 GPU tensor (binary searches on the GPU). selectivity=1:
    bit-exact create_relation_zipf; < 1: this build's selectivity extension (BASELINE config 5)."""
    _err(lib().hwbrj_create_relation_zipf_device(_ptr(out), out.shape[0], alphabet_size, theta,
                                                 seed, selectivity, host_threads, None),
         "hwbrj_create_relation_zipf_device")


def rand_stream(seed: int, n: int) -> np.ndarray:
    """The first n values of glibc rand() after srand(seed), from the library's restatement."""
    out = np.empty(n, dtype=np.int32)
    _err(lib().hwbrj_rand_stream(seed, out.ctypes.data, n), "hwbrj_rand_stream")
    return out


def reference_relations(r_size: int, s_size: int, selectivity: float = 1.0, skew: float = 0.0,
                        non_unique: bool = False, full_range: bool = False, r_seed: int = 12345,
                        s_seed: int = 54321, nthreads: int = 2, host_threads: int = 0):
    """(R, S) as the reference's main() builds them (src/main.c:410-466), on the host:
    --full-range, --non-unique and -z are bit-exact (keys and order) to the reference for the same
    seeds; the default PK/FK relations have the reference's key multiset in a seeded order."""
    if full_range or non_unique:
        thr = nonunique_threshold(r_size, selectivity, full_range)
        R = create_relation_nonunique(r_size, thr, r_seed)
        mk = create_relation_fk_from_pk if full_range else create_relation_nonunique_from_pk
        return R, mk(s_size, R, thr, selectivity, s_seed)
    R = generate_host(r_size, nthreads, r_size, r_size, 1.0, r_seed, host_threads)
    if skew > 0:
        return R, create_relation_zipf(s_size, r_size, skew, s_seed, host_threads)
    return R, generate_host(s_size, nthreads, 2**31 - 1, r_size, selectivity, s_seed, host_threads)


def export_filter(m_bits: int) -> np.ndarray:
    """The last join's filter in the reference's byte layout (m/8 uint8)."""
    out = np.empty(m_bits // 8, dtype=np.uint8)
    _err(lib().hwbrj_export_filter(out.ctypes.data, out.nbytes), "hwbrj_export_filter")
    return out


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Rows [lo, hi) of an n-row relation owned by `rank` of `world` (range sharding of S, the
    multi-GPU analogue of the reference's per-thread chunking,
    src/parallel_radix_join_bloom.c:1646-1670: equal chunks, the remainder spread evenly)."""
    return rank * n // world, (rank + 1) * n // world


def hash_crc(seed: int, key: int) -> int:
    return lib().hwbrj_hash_crc(seed, key)


def hash_crapwow(seed: int, key: int) -> int:
    return lib().hwbrj_hash_crapwow(seed, key)
