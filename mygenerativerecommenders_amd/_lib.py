"""Loader for the gfx950 C-ABI library ``libgr_hstu.so``.

The ctypes signatures are derived from ``include/gr_hstu.h`` itself, so the Python
side and the C-ABI cannot drift.  There is no fallback: if the library or a GPU is
missing, every op raises.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import re
import threading

import torch  # noqa: F401  (import first: its HIP runtime is the one the .so binds to)

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
# GR_HSTU_LIB selects an alternative build of the same library (kernel experiments).
LIB_PATH = os.environ.get("GR_HSTU_LIB") or os.path.join(PKG_DIR, "libgr_hstu.so")
HEADER_PATH = os.path.join(REPO_DIR, "include", "gr_hstu.h")

_CTYPES = {
    "void": None,
    "int": ctypes.c_int,
    "int64_t": ctypes.c_int64,
    "uint64_t": ctypes.c_uint64,
    "size_t": ctypes.c_size_t,
    "float": ctypes.c_float,
    "double": ctypes.c_double,
    "const char*": ctypes.c_char_p,
}

_lock = threading.Lock()
_lib = None


def parse_header(path: str = HEADER_PATH):
    """Returns {name: (restype_str, [argtype_str, ...])} for every GR_API function."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    out = {}
    for m in re.finditer(r"GR_API\s+([\w\s\*]+?)\s*\b(\w+)\s*\(([^)]*)\)\s*;", text, flags=re.S):
        ret, name, args = m.group(1).strip(), m.group(2), m.group(3).strip()
        types = []
        if args and args != "void":
            for a in args.split(","):
                a = " ".join(a.split())
                a = re.sub(r"\s*\*\s*", "* ", a).strip()
                # drop the parameter name
                t = a.rsplit(" ", 1)[0] if " " in a else a
                types.append(t.replace("* ", "*").strip())
        out[name] = (ret.replace(" *", "*"), types)
    return out


def _ctype(t: str):
    t = t.strip()
    if t in _CTYPES:
        return _CTYPES[t]
    if t.endswith("*"):
        return ctypes.c_void_p
    raise TypeError(f"unmapped C type {t!r} in gr_hstu.h")


def lib():
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; "
                "g.build()'` (hipcc --offload-arch=gfx950). There is no CPU fallback.")
        L = ctypes.CDLL(LIB_PATH)
        for name, (ret, args) in parse_header().items():
            fn = getattr(L, name)
            fn.restype = _ctype(ret) if ret != "void" else None
            fn.argtypes = [_ctype(a) for a in args]
        _lib = L
    return _lib


class GrError(RuntimeError):
    pass


def call(name: str, *args):
    """Calls a C-ABI entry point; raises GrError(gr_last_error()) on non-zero status.

    The argument count must equal the header's: ctypes would pass surplus arguments as
    varargs, so a caller written against another ABI version would shift every later
    pointer and size silently.
    """
    L = lib()
    fn = getattr(L, name)
    if len(args) != len(fn.argtypes):
        raise GrError(f"{name} takes {len(fn.argtypes)} arguments (gr_hstu.h, ABI "
                      f"{L.gr_version()}), got {len(args)}")
    rc = fn(*args)
    if rc != 0:
        msg = L.gr_last_error().decode(errors="replace")
        raise GrError(f"{name} failed (status {rc}): {msg}")


KERNEL_NAMES = ("bucket_map", "attn_fwd", "attn_bwd", "attn_bwd_dkv", "attn_bwd_dq", "attn_bias_reduce", "attn_bf16_copies",
                "weight_images",
                "attn_fwd_bnd", "attn_fwd_bnd1", "attn_bwd_dq_bnd", "attn_bwd_dq_bnd1",
                "ln_uvqk_fwd", "gate_o_fwd", "gate_o_bwd", "ln_uvqk_bwd", "boundary_fwd", "boundary_bwd",
                "wgrad_partial",
                "wgrad_reduce", "mips_pack", "mips_select", "mips_merge", "mips_small", "mips_sample", "mips_tau",
                "mips_filter", "mips_select_fallback", "mips_merge_fallback", "cumsum", "encoder_prologue", "bf16_scale_add", "adamw",
                "dense_to_jagged", "jagged_to_padded", "l2_normalize", "current_embeddings",
                "sampled_softmax_fwd", "sampled_softmax_bwd", "sampled_softmax_csr",
                "sampled_softmax_table_grad", "preproc", "item_embedding", "mips_sort_invalid",
                "mips_wide_score", "mips_wide_select", "rows_copy", "decode_scatter", "decode_attn",
                "softmax_attn_fwd", "softmax_attn_bwd", "rel_bias_fwd", "rel_bias_bwd")


def parse_options(path: str = HEADER_PATH) -> dict:
    """{"MIPS_FILTER_FP32": 1, ...}: the GR_OPT_* launch options declared in gr_hstu.h."""
    text = re.sub(r"/\*.*?\*/", "", open(path).read(), flags=re.S)  # the enum, not the comments
    return {m.group(1): int(m.group(2))
            for m in re.finditer(r"\bGR_OPT_([A-Z0-9_]*[A-Z0-9])\s*=\s*(\d+)", text)}


def set_option(name: str, value: int) -> int:
    """Sets launch option GR_OPT_<name>; returns the previous value."""
    opt = parse_options()[name]
    L = lib()
    old = L.gr_get_option(opt)
    call("gr_set_option", opt, int(value))
    return old


def get_option(name: str) -> int:
    return lib().gr_get_option(parse_options()[name])


@contextlib.contextmanager
def option(name: str, value: int):
    """Scoped launch option (tests, A/B measurements)."""
    old = set_option(name, value)
    try:
        yield
    finally:
        set_option(name, old)


def set_thread_option(name: str, value: int) -> None:
    """Overrides launch option GR_OPT_<name> for the calling thread only (gr_set_thread_option);
    launches and workspace queries from other threads keep their own values."""
    call("gr_set_thread_option", parse_options()[name], int(value))


def clear_thread_option(name: str | None = None) -> None:
    """Drops the calling thread's override of GR_OPT_<name> (all overrides for None)."""
    call("gr_clear_thread_option", 0 if name is None else parse_options()[name])


@contextlib.contextmanager
def thread_option(name: str, value: int):
    """Scoped per-thread launch option.  Note that torch runs autograd backward functions
    of GPU tensors on its own device threads: options meant for a backward must be
    process-wide (``option``) or set inside the backward's thread."""
    set_thread_option(name, value)
    try:
        yield
    finally:
        clear_thread_option(name)


def timing_enable(on: bool = True):
    """Library-level live kernel timing (HIP event pair around every launch)."""
    lib().gr_timing_enable(1 if on else 0)


def kernel_times(names=KERNEL_NAMES) -> dict:
    """Drains the recorded event pairs: {kernel: (total_ms, launches)}."""
    L = lib()
    out = {}
    for n in names:
        ms = ctypes.c_double(0.0)
        cnt = ctypes.c_int(0)
        rc = L.gr_timing_query(n.encode(), ctypes.byref(ms), ctypes.byref(cnt))
        if rc != 0:
            raise GrError(L.gr_last_error().decode())
        out[n] = (ms.value, cnt.value)
    return out


def ptr(t) -> int | None:
    """Device pointer of a tensor (None for None)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(device=None) -> int:
    import torch as _t
    return _t.cuda.current_stream(device).cuda_stream


def require_gpu(*tensors):
    import torch as _t
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise GrError("gr_hstu ops run on the MI355X only: got a CPU tensor "
                          "(the CPU restatement lives in oracle/ and is test-only)")
    if not _t.cuda.is_available():
        raise GrError("no GPU visible: gr_hstu has no CPU path")
