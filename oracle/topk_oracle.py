"""ctypes wrapper for the C top-k oracle (``topk_oracle.c``) — TEST INFRASTRUCTURE
ONLY (tests/, smoke(), bench.py cpu_baseline).  See the C file's header for the
reference lines it restates."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libgr_oracle.so")
_lib = None


def build() -> str:
    src = os.path.join(HERE, "topk_oracle.c")
    if (not os.path.exists(LIB_PATH)) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", HERE, "libgr_oracle.so"])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        L.gr_oracle_mips_topk.argtypes = [P, P, P, P, ctypes.c_int, ctypes.c_int64,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, P]
        L.gr_oracle_mips_topk.restype = ctypes.c_int
        L.gr_oracle_scores.argtypes = [P, P, ctypes.c_int, ctypes.c_int64, ctypes.c_int, P]
        L.gr_oracle_scores.restype = None
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def mips_topk(Q: np.ndarray, E: np.ndarray, item_ids: np.ndarray | None,
              invalid: np.ndarray | None, k: int):
    """Returns (scores (B,k) f32, ids (B,k) i64, idx (B,k) i64), canonical order."""
    Q = np.ascontiguousarray(Q, dtype=np.float32)
    E = np.ascontiguousarray(E, dtype=np.float32)
    B, D = Q.shape
    X = E.shape[0]
    ids = None if item_ids is None else np.ascontiguousarray(item_ids, dtype=np.int64).reshape(-1)
    inv = None if invalid is None else np.ascontiguousarray(invalid, dtype=np.int64)
    N0 = 0 if inv is None else inv.shape[1]
    s = np.empty((B, k), np.float32)
    o_ids = np.empty((B, k), np.int64)
    o_idx = np.empty((B, k), np.int64)
    rc = lib().gr_oracle_mips_topk(_ptr(Q), _ptr(E), _ptr(ids), _ptr(inv), B, X, D, N0, k,
                                   _ptr(s), _ptr(o_ids), _ptr(o_idx))
    if rc != 0:
        raise RuntimeError(f"gr_oracle_mips_topk failed: {rc}")
    return s, o_ids, o_idx


def scores(Q: np.ndarray, E: np.ndarray) -> np.ndarray:
    Q = np.ascontiguousarray(Q, dtype=np.float32)
    E = np.ascontiguousarray(E, dtype=np.float32)
    out = np.empty((Q.shape[0], E.shape[0]), np.float32)
    lib().gr_oracle_scores(_ptr(Q), _ptr(E), Q.shape[0], E.shape[0], Q.shape[1], _ptr(out))
    return out
