"""ctypes access to the oracle (TEST INFRASTRUCTURE ONLY -- see oracle.h).

  liboracle.so        C restatement of the reference BPRO path (oracle.c)
  _ref/libbloomref.so the reference's own src/hash.c + src/bloom_filter.c, compiled unmodified

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
REFLIB = os.path.join(HERE, "_ref", "libbloomref.so")

_L = None
_R = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib() -> ctypes.CDLL:
    global _L
    if _L is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        L.orc_crc32c.restype = ctypes.c_uint32
        L.orc_crc32c.argtypes = [ctypes.c_uint32, ctypes.c_int32]
        L.orc_crapwow.restype = ctypes.c_uint32
        L.orc_crapwow.argtypes = [ctypes.c_uint32, ctypes.c_int32]
        L.orc_gen_keys.restype = ctypes.c_int
        L.orc_gen_keys.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                   ctypes.c_uint64, ctypes.c_uint64, ctypes.c_double]
        L.orc_shuffle_keys.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64]
        L.orc_bpro.restype = ctypes.c_int64
        L.orc_bpro.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                               ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
                               ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64),
                               ctypes.c_void_p]
        L.orc_bloom_init.restype = ctypes.c_int
        L.orc_bloom_init.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64,
                                     ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32]
        L.orc_bloom_free.argtypes = [ctypes.c_void_p]
        L.orc_bloom_add_all.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
        L.orc_bloom_add_all_atomic.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
        L.orc_count_filtered.restype = ctypes.c_uint64
        L.orc_count_filtered.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
        L.orc_bloom_popcount.restype = ctypes.c_uint64
        L.orc_bloom_popcount.argtypes = [ctypes.c_void_p]
        L.orc_bloom_args_invalid.restype = ctypes.c_int
        L.orc_bloom_args_invalid.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64]
        L.orc_gen_nonunique.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int64,
                                        ctypes.c_uint32]
        for fn in (L.orc_gen_nonunique_from_pk, L.orc_gen_fk_from_pk):
            fn.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                           ctypes.c_int64, ctypes.c_double, ctypes.c_uint32]
        L.orc_gen_zipf.restype = ctypes.c_int
        L.orc_gen_zipf.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint, ctypes.c_double,
                                   ctypes.c_uint32]
        L.orc_join_pairs.restype = ctypes.c_int64
        L.orc_join_pairs.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                     ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64]
        L.orc_fpr_test.restype = ctypes.c_int
        L.orc_fpr_test.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                   ctypes.c_uint32, ctypes.c_void_p]
        _L = L
    return _L


def fpr_test(seed: int, m: int, kmax: int, n_samples: int, n_insertions: int):
    """The reference's FPR unit test (src/unit_tests.c:191-283): ({k: fpr_emp %} blocked B=512,
    {k: fpr_emp %} basic), fpr_emp = false positives / n_samples."""
    pos = np.zeros(2 * kmax, dtype=np.uint64)
    if lib().orc_fpr_test(seed, m, kmax, n_samples, n_insertions, pos.ctypes.data):
        raise MemoryError
    pct = pos.astype(np.float64) / n_samples * 100.0
    return ({k + 1: pct[k] for k in range(kmax)}, {k + 1: pct[kmax + k] for k in range(kmax)})


def join_pairs(R: np.ndarray, S: np.ndarray) -> np.ndarray:
    """(n, 2) int32 {R.payload, S.payload} of every match (JOIN_RESULT_MATERIALIZE), unordered."""
    R = np.ascontiguousarray(R, dtype=np.int32)
    S = np.ascontiguousarray(S, dtype=np.int32)
    n = lib().orc_join_pairs(R.ctypes.data, R.shape[0], S.ctypes.data, S.shape[0], None, 0)
    if n < 0:
        raise MemoryError
    out = np.empty((n, 2), dtype=np.int32)
    lib().orc_join_pairs(R.ctypes.data, R.shape[0], S.ctypes.data, S.shape[0], out.ctypes.data, n)
    return out


def threshold(r_size: int, q: float, full_range: bool) -> int:
    """src/main.c:421-427."""
    import math
    t = math.ceil(2147483647 * q)
    return t if full_range else int(min(r_size, t))


def reference_relations(r_size: int, s_size: int, q: float, mode: str, skew: float = 0.0,
                        r_seed: int = 12345, s_seed: int = 54321):
    """(R, S) of src/main.c:410-466 for mode 'nonunique' | 'fullrange' | 'zipf', drawn with libc
    rand() itself. zipf: R = keys 1..r_size in order (its order does not matter)."""
    L = lib()
    R = np.empty((r_size, 2), dtype=np.int32)
    S = np.empty((s_size, 2), dtype=np.int32)
    if mode == "zipf":
        R[:, 0] = np.arange(1, r_size + 1)
        R[:, 1] = np.arange(r_size)
        if L.orc_gen_zipf(S.ctypes.data, s_size, r_size, skew, s_seed):
            raise MemoryError
        return R, S
    thr = threshold(r_size, q, mode == "fullrange")
    L.orc_gen_nonunique(R.ctypes.data, r_size, thr, r_seed)
    fn = L.orc_gen_fk_from_pk if mode == "fullrange" else L.orc_gen_nonunique_from_pk
    fn(S.ctypes.data, s_size, R.ctypes.data, r_size, thr, q, s_seed)
    return R, S


class _Bloom(ctypes.Structure):  # orc_bloom_t
    _fields_ = [("variant", ctypes.c_int), ("seed", ctypes.c_uint32), ("m", ctypes.c_uint64),
                ("k", ctypes.c_uint64), ("B", ctypes.c_uint64), ("nblocks", ctypes.c_uint64),
                ("bitmap", ctypes.POINTER(ctypes.c_uint8))]


class _Timing(ctypes.Structure):
    _fields_ = [("total_usec", ctypes.c_double), ("partition_usec", ctypes.c_double),
                ("join_usec", ctypes.c_double), ("phase_usec", ctypes.c_double * 6)]


def crc(seed: int, key: int) -> int:
    return lib().orc_crc32c(seed, key)


def crapwow(seed: int, key: int) -> int:
    return lib().orc_crapwow(seed, key)


def gen_keys(n: int, nthreads: int, maxid: int, threshold: int, q: float,
             shuffle_seed: int | None = None) -> np.ndarray:
    """Reference key multiset (src/generator.c:304-415), generation order unless shuffled."""
    k = np.empty(n, dtype=np.int32)
    rc = lib().orc_gen_keys(k.ctypes.data, n, nthreads, maxid, threshold, q)
    if rc:
        raise ValueError(f"orc_gen_keys rc={rc}")
    if shuffle_seed is not None:
        lib().orc_shuffle_keys(k.ctypes.data, n, shuffle_seed)
    return k


def relation(n: int, nthreads: int, maxid: int, threshold: int, q: float, seed: int) -> np.ndarray:
    """(n, 2) int32 {key, payload=row} with a seeded shuffle of the keys (reference layout)."""
    t = np.empty((n, 2), dtype=np.int32)
    t[:, 0] = gen_keys(n, nthreads, maxid, threshold, q, seed)
    t[:, 1] = np.arange(n, dtype=np.int64).astype(np.int32)
    return t


def bpro(R: np.ndarray, S: np.ndarray, nthreads: int = 8, variant: int = 1, m: int = 0,
         k: int = 1, B: int = 1024, use_bloom: bool = True):
    """(matches, filtered, timing_usec) of the oracle's multithreaded BPRO/PRO restatement."""
    R = np.ascontiguousarray(R, dtype=np.int32)
    S = np.ascontiguousarray(S, dtype=np.int32)
    f = ctypes.c_uint64()
    tm = _Timing()
    res = lib().orc_bpro(R.ctypes.data, R.shape[0], S.ctypes.data, S.shape[0], nthreads, variant,
                         m, k, B, 1 if use_bloom else 0, ctypes.byref(f), ctypes.byref(tm))
    if res < 0:
        raise MemoryError("orc_bpro allocation failed")
    return int(res), int(f.value), {"total": tm.total_usec, "partition": tm.partition_usec,
                                    "join": tm.join_usec, "phases": list(tm.phase_usec)}


def bloom_bitmap(keys: np.ndarray, variant: int, m: int, k: int, B: int):
    """(bitmap bytes, popcount) after inserting keys with the oracle's filter (seed 42)."""
    f = _Bloom()
    keys = np.ascontiguousarray(keys, dtype=np.int32)
    if lib().orc_bloom_init(ctypes.byref(f), variant, m, k, B, 42):
        raise MemoryError
    lib().orc_bloom_add_all(ctypes.byref(f), keys.ctypes.data, keys.shape[0])
    bm = np.ctypeslib.as_array(f.bitmap, shape=(m // 8,)).copy()
    pc = lib().orc_bloom_popcount(ctypes.byref(f))
    lib().orc_bloom_free(ctypes.byref(f))
    return bm, int(pc)


def count_filtered(R_keys: np.ndarray, S_keys: np.ndarray, variant: int, m: int, k: int, B: int) -> int:
    f = _Bloom()
    R_keys = np.ascontiguousarray(R_keys, dtype=np.int32)
    S_keys = np.ascontiguousarray(S_keys, dtype=np.int32)
    if lib().orc_bloom_init(ctypes.byref(f), variant, m, k, B, 42):
        raise MemoryError
    lib().orc_bloom_add_all(ctypes.byref(f), R_keys.ctypes.data, R_keys.shape[0])
    c = lib().orc_count_filtered(ctypes.byref(f), S_keys.ctypes.data, S_keys.shape[0])
    lib().orc_bloom_free(ctypes.byref(f))
    return int(c)


# ------------------------------------------------------------------ the reference itself
class _RefFilter(ctypes.Structure):  # src/bloom_filter.h:12-20
    _fields_ = [("variant", ctypes.c_int), ("bitmap", ctypes.POINTER(ctypes.c_uint8)),
                ("seed", ctypes.c_uint32), ("m", ctypes.c_uint64), ("k", ctypes.c_uint64),
                ("B", ctypes.c_uint64), ("nblocks", ctypes.c_uint64)]


_ADD = ctypes.CFUNCTYPE(None, ctypes.POINTER(_RefFilter), ctypes.c_int32)
_CONTAINS = ctypes.CFUNCTYPE(ctypes.c_bool, ctypes.POINTER(_RefFilter), ctypes.c_int32)


class _RefStrategy(ctypes.Structure):  # src/bloom_filter.h:43-48
    _fields_ = [("variant", ctypes.c_int), ("filter", ctypes.POINTER(_RefFilter)),
                ("add", _ADD), ("contains", _CONTAINS)]


class _RefArgs(ctypes.Structure):  # src/bloom_filter.h:50-55
    _fields_ = [("variant", ctypes.c_int), ("m", ctypes.c_uint64), ("k", ctypes.c_uint64),
                ("B", ctypes.c_uint64)]


def have_ref() -> bool:
    return os.path.exists(REFLIB)


def ref() -> ctypes.CDLL:
    global _R
    if _R is None:
        R = ctypes.CDLL(REFLIB)
        R.hash_crc.restype = ctypes.c_uint32
        R.hash_crc.argtypes = [ctypes.c_uint32, ctypes.c_int32]
        R.hash_crapwow.restype = ctypes.c_uint32
        R.hash_crapwow.argtypes = [ctypes.c_uint32, ctypes.c_int32]
        R.bloom_filter_create.restype = ctypes.POINTER(_RefStrategy)
        R.bloom_filter_create.argtypes = [ctypes.POINTER(_RefArgs), ctypes.c_uint32]
        R.bloom_filter_destroy.argtypes = [ctypes.POINTER(_RefStrategy)]
        R.ref_add_all.argtypes = [ctypes.POINTER(_RefStrategy), ctypes.c_void_p, ctypes.c_uint64]
        R.ref_count.restype = ctypes.c_uint64
        R.ref_count.argtypes = [ctypes.POINTER(_RefStrategy), ctypes.c_void_p, ctypes.c_uint64]
        _R = R
    return _R


def ref_bloom(keys_build: np.ndarray, keys_probe: np.ndarray | None, variant: int, m: int, k: int,
              B: int):
    """Run the reference's own bloom_filter.c (seed 42): (bitmap bytes, filtered count)."""
    a = _RefArgs(variant, m, k, B)
    st = ref().bloom_filter_create(ctypes.byref(a), 42)
    s = st.contents
    kb = np.ascontiguousarray(keys_build, dtype=np.int32)
    ref().ref_add_all(st, kb.ctypes.data, kb.shape[0])
    cnt = None
    if keys_probe is not None:
        kp = np.ascontiguousarray(keys_probe, dtype=np.int32)
        cnt = int(ref().ref_count(st, kp.ctypes.data, kp.shape[0]))
    bm = np.ctypeslib.as_array(s.filter.contents.bitmap, shape=(m // 8,)).copy()
    ref().bloom_filter_destroy(st)
    return bm, cnt
