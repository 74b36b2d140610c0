"""ctypes wrapper of the CPU checker libraries — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module; the product (foundationdb_amd) never does.

* ``OracleConflictSet`` wraps semantic_oracle.cpp, the restatement of
  fdbserver/SkipList.cpp semantics used as the parity checker.
* ``SkipListBaseline`` wraps skiplist_baseline.cpp, the performance-faithful
  restatement of the reference skip list timed as the CPU baseline.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIBS = {}


def build(force: bool = False) -> None:
    """make is incremental: rebuilds a checker library only when its sources changed."""
    if force:
        subprocess.check_call(["make", "-s", "-C", HERE, "clean"])
    subprocess.check_call(["make", "-s", "-C", HERE, "all"])


def _lib(name: str):
    if name not in _LIBS:
        path = os.path.join(HERE, name)
        if not os.path.exists(path):
            build()
        _LIBS[name] = ctypes.CDLL(path)
    return _LIBS[name]


def _p(a):
    return ctypes.c_void_p(a.ctypes.data if a.size else 0)


class _CSBase:
    """Shared ctypes plumbing: both checker libraries export the same C surface with a prefix."""

    _libname = ""
    _prefix = ""

    def __init__(self):
        L = _lib(self._libname)
        self._L = L
        pre = self._prefix
        self._fn = {}
        for n, res, args in [
            ("new", ctypes.c_void_p, []),
            ("destroy", None, [ctypes.c_void_p]),
            ("clear", None, [ctypes.c_void_p, ctypes.c_int64]),
            ("set_oldest", None, [ctypes.c_void_p, ctypes.c_int64]),
            ("oldest", ctypes.c_int64, [ctypes.c_void_p]),
            ("history_size", ctypes.c_int64, [ctypes.c_void_p]),
            (
                "load_history",
                None,
                [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64],
            ),
            (
                "detect",
                ctypes.c_int64,
                [
                    ctypes.c_void_p,
                    ctypes.c_void_p,
                    ctypes.c_int64,
                    ctypes.c_int64,
                    ctypes.c_void_p,
                    ctypes.c_void_p,
                    ctypes.c_void_p,
                    ctypes.c_int64,
                    ctypes.c_int,
                ],
            ),
        ]:
            f = getattr(L, pre + n)
            f.restype = res
            f.argtypes = args
            self._fn[n] = f
        self._h = self._fn["new"]()
        self._last_T = 0

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._fn["destroy"](h)
            self._h = None

    def clear(self, version: int) -> None:
        self._fn["clear"](self._h, version)

    def set_oldest_version(self, v: int) -> None:
        self._fn["set_oldest"](self._h, v)

    @property
    def oldest_version(self) -> int:
        return self._fn["oldest"](self._h)

    def history_size(self) -> int:
        return self._fn["history_size"](self._h)

    def load_history(self, key_bytes, key_offsets, versions, header_version: int = 0) -> None:
        kb = np.ascontiguousarray(key_bytes, np.uint8)
        ko = np.ascontiguousarray(key_offsets, np.int64)
        vv = np.ascontiguousarray(versions, np.int64)
        self._fn["load_history"](self._h, len(vv), _p(kb), _p(ko), _p(vv), header_version)

    def detect(self, pb, now: int, new_oldest: int, gc=True, add_oldest=None):
        """Returns (verdicts uint8[T], conflicting: dict txn -> sorted list of read indices).

        gc: False = no removeBefore; True = a full removeBefore pass (history size comparable with
        the GPU engine after its full GC); "bounded" = the reference's bounded, resumable
        removeBefore (SkipList.cpp:880-889; the skip-list restatement only).
        add_oldest: the oldestVersion the batch's addTransaction saw when the caller added it
        before the previous batch's detect (SkipList.cpp:770 reads it at add); None = added right
        before this detect, as the Resolver does (Resolver.actor.cpp:179-194)."""
        if add_oldest is not None:
            f = getattr(self._L, self._prefix + "set_add_oldest")
            f.restype = None
            f.argtypes = [ctypes.c_void_p, ctypes.c_int64]
            f(self._h, int(add_oldest))
        T = pb.n_txn
        verdicts = np.zeros(T, np.uint8)
        cap = max(1, pb.n_reads)
        off = np.zeros(T + 1, np.int32)
        idx = np.zeros(cap, np.int32)
        cs = pb.c_struct()
        n = self._fn["detect"](
            self._h, ctypes.byref(cs), now, new_oldest, _p(verdicts), _p(off), _p(idx), cap,
            2 if gc == "bounded" else (1 if gc else 0)
        )
        if n < 0:
            raise RuntimeError("oracle detect failed")
        self._last_T = T
        # conflictingKeyRangeMap as the reference fills it: an entry for every reporting transaction
        # that was admitted with at least one read range (created in addTransaction,
        # SkipList.cpp:777-784), holding the conflicting read indices (empty if it committed)
        conf = {}
        roff = pb.read_offsets
        for t in range(T):
            if pb.report[t] and roff[t + 1] > roff[t] and verdicts[t] != 1:
                conf[t] = idx[off[t] : off[t + 1]].tolist()
        return verdicts, conf


class OracleConflictSet(_CSBase):
    _libname = "liboracle.so"
    _prefix = "oracle_"

    def version_at(self, key: bytes) -> int:
        f = self._L.oracle_version_at
        f.restype = ctypes.c_int64
        f.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int64]
        return f(self._h, key, len(key))

    def last_lists(self, with_too_old: bool):
        """(nonConflicting, tooOld) of the last detect, as SkipList.cpp:869-876 fills them when the
        caller passes a tooOld list (with_too_old) or nullptr; tooOld is None in the second case."""
        f = self._L.oracle_last_lists
        f.restype = None
        f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                      ctypes.c_void_p]
        cap = max(1, self._last_T)
        nc, to = np.zeros(cap, np.int32), np.zeros(cap, np.int32)
        n_nc, n_to = np.zeros(1, np.int32), np.zeros(1, np.int32)
        f(self._h, int(bool(with_too_old)), _p(nc), _p(n_nc), _p(to), _p(n_to))
        return nc[: n_nc[0]].tolist(), (to[: n_to[0]].tolist() if with_too_old else None)

    def dump_history(self):
        n = self.history_size()
        cap_bytes = max(1, n * 64)
        while True:
            kb = np.zeros(cap_bytes, np.uint8)
            ko = np.zeros(n + 1, np.int64)
            vv = np.zeros(max(1, n), np.int64)
            f = self._L.oracle_dump_history
            f.restype = ctypes.c_int64
            f.argtypes = [ctypes.c_void_p] + [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_int64]
            got = f(self._h, _p(kb), cap_bytes, _p(ko), _p(vv), n)
            if got >= 0:
                keys = [kb[ko[i] : ko[i + 1]].tobytes() for i in range(got)]
                return keys, vv[:got].copy()
            cap_bytes *= 4


class SkipListBaseline(_CSBase):
    _libname = "libskiplist_baseline.so"
    _prefix = "slb_"

    PHASES = ("add", "sort", "check_read", "intra", "combine", "merge", "remove_before", "total")

    def last_times(self) -> dict:
        """Seconds per phase of the last detect (the reference's PerfDoubleCounters, SkipList.cpp:49-51)."""
        f = self._L.slb_last_times
        f.restype = None
        f.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        out = np.zeros(8, np.float64)
        f(self._h, _p(out))
        return dict(zip(self.PHASES, out.tolist()))


def point_compare(a: bytes, a_begin: bool, a_write: bool, b: bytes, b_begin: bool, b_write: bool) -> int:
    f = _lib("liboracle.so").oracle_point_compare
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int] * 2
    return f(a, len(a), int(a_begin), int(a_write), b, len(b), int(b_begin), int(b_write))
