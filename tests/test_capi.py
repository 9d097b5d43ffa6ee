"""CPU: the C-ABI library loads, exports exactly what include/gr_hstu.h declares, and
follows the error convention (non-zero status + thread-local gr_last_error) — all
without touching a GPU (argument validation runs before any HIP call)."""
import ctypes
import os
import re
import subprocess

import pytest

from mygenerativerecommenders_amd import _lib


def test_library_loads_and_version():
    L = _lib.lib()
    hdr = open(_lib.HEADER_PATH).read()
    ver = int(re.search(r"#define GR_HSTU_ABI_VERSION (\d+)", hdr).group(1))
    assert L.gr_version() == ver


def test_exports_match_header():
    decl = set(_lib.parse_header())
    assert len(decl) >= 19
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = decl - exported
    assert not missing, f"declared but not exported: {missing}"
    extra = {e for e in exported if not e.startswith("_")} - decl
    assert not extra, f"exported but not declared: {extra}"


def test_every_declared_symbol_resolves_with_signature():
    L = _lib.lib()
    for name, (ret, args) in _lib.parse_header().items():
        fn = getattr(L, name)
        assert len(fn.argtypes) == len(args), name


@pytest.mark.parametrize("name,nargs", [("hstu_attn_fwd", 19), ("mips_topk", 16),
                                        ("hstu_ln_uvqk_fwd", 15), ("gr_wgrad", 15)])
def test_null_pointer_is_an_error_not_a_crash(name, nargs):
    L = _lib.lib()
    _, args = _lib.parse_header()[name]
    assert len(args) == nargs
    vals = []
    for a in args:
        vals.append(None if a.endswith("*") else 1)
    rc = getattr(L, name)(*vals)
    assert rc != 0
    msg = L.gr_last_error().decode()
    assert name.split("_")[0] in msg or "null" in msg or "bad" in msg


def test_error_is_raised_as_python_exception():
    _, args = _lib.parse_header()["hstu_attn_fwd"]
    vals = [None if a.endswith("*") else 1 for a in args]
    with pytest.raises(_lib.GrError, match="hstu_attn_fwd"):
        _lib.call("hstu_attn_fwd", *vals)


def test_call_rejects_wrong_argument_count():
    """ctypes passes surplus arguments as varargs; _lib.call must refuse them (and short
    lists) before anything reaches the library."""
    _, args = _lib.parse_header()["hstu_attn_fwd"]
    vals = [None if a.endswith("*") else 1 for a in args]
    with pytest.raises(_lib.GrError, match="takes 19 arguments"):
        _lib.call("hstu_attn_fwd", *vals, 0)
    with pytest.raises(_lib.GrError, match="takes 19 arguments"):
        _lib.call("hstu_attn_fwd", *vals[:-1])
    with pytest.raises(_lib.GrError, match="got 0"):
        _lib.call("gr_wgrad")


def test_workspace_size_queries_are_host_only():
    L = _lib.lib()
    slabs = 4 * 128 * 4 * (2 * 211 - 1 + 129)
    ds = 4 * 256 * 14 * 15 // 2 * 128  # dS tiles of the two-pass backward (N <= 512, default)
    assert L.hstu_attn_bwd_workspace_size(128, 211, 200, 1, 128) == (slabs + 255) // 256 * 256 + ds
    with _lib.option("ATTN_BWD_DS", 0):
        assert L.hstu_attn_bwd_workspace_size(128, 211, 200, 1, 128) == slabs
    slabs3 = 4 * 32 * 32 * (2 * 2059 - 1 + 129)
    assert L.hstu_attn_bwd_workspace_size(32, 2059, 2048, 1, 128) == slabs3  # no dS above 512
    # head dims given: narrow heads as above; wide heads (d > 128) add the dS tiles at any N
    assert L.hstu_attn_bwd_workspace_size_d(32, 2059, 2048, 1, 64, 64, 128) == slabs3
    ds3 = 4 * 256 * 129 * 130 // 2 * 32
    assert L.hstu_attn_bwd_workspace_size_d(32, 2059, 2048, 1, 256, 256, 128) == \
        (slabs3 + 255) // 256 * 256 + ds3
    with _lib.option("ATTN_BWD_WIDE_DS", 0):
        assert L.hstu_attn_bwd_workspace_size_d(32, 2059, 2048, 1, 256, 256, 128) == slabs3
    assert L.hstu_bucket_map_bytes(128, 211) == 2 * 128 * 10 * 4096
    assert L.mips_packed_items_bytes(3953, 50) == 4 * ((3953 + 15) // 16) * 7 * 128
    # filter-sized catalogs: f32 blocks | bf16 copy (a full 16x16x32 chunk + 2 of the second
    # chunk's 4 lane groups + a 64-byte tail for dims 48, 49 = 1,600 B per 16 items) |
    # max norm | row-major f32 rows padded to 52 floats
    X = 1_000_003
    nblk = (X + 15) // 16
    f32 = 4 * nblk * 7 * 128
    al = lambda v: (v + 255) // 256 * 256  # noqa: E731
    assert L.mips_packed_items_bytes(X, 50) == (al(f32) + al(nblk * 1600) + 256
                                                + al(4 * X * 52))
    # D = 52: the last group holds 4 dims (no tail; 1,792 B)
    assert L.mips_packed_items_bytes(X, 52) == (al(f32) + al(nblk * 1792) + 256
                                                + al(4 * X * 52))
    assert L.mips_packed_items_bytes(X, 64) == (al(4 * nblk * 8 * 128) + al(nblk * 2048) + 256
                                                + al(4 * X * 64))
    # D = 65: three k-chunks, the last with one stored lane group (2,304 B per 16 items)
    assert L.mips_packed_items_bytes(X, 65) == (al(4 * nblk * 9 * 128) + al(nblk * 2304) + 256
                                                + al(4 * X * 68))
    assert L.mips_packed_items_bytes(X, 257) == 4 * nblk * 33 * 128  # D > 256: no filter copy
    assert L.gr_wgrad_workspace_size(27008, 50, 200) > 0
    assert L.mips_topk_workspace_size(128, 10_000_000, 50, 200, 211) > 0
    assert L.mips_topk_workspace_size(128, 27_278, 50, 200, 2059) > L.mips_topk_workspace_size(128, 27_278, 50, 200, 211)
    assert L.mips_topk_workspace_size(128, 3953, 50, 2259, 0) > 0
    assert L.hstu_attn_bwd_workspace_size(0, 211, 200, 1, 128) == 0


def test_option_changed_between_sizing_and_launch_is_rejected():
    """A launch re-derives its workspace need under the options in force at launch time
    and returns non-zero when the caller's workspace (sized under other options) is
    smaller — never an overflow.  The check runs before any device work, so fake
    non-null pointers are safe here (no GPU needed)."""
    L = _lib.lib()
    fake = 1 << 20  # never dereferenced: the launch returns at the workspace check
    # Ka = 300 (> 256: the narrow plan only, whose split size the option sets)
    with _lib.option("WGRAD_ROWS", 4096):
        ws = L.gr_wgrad_workspace_size(200000, 300, 200)
    with _lib.option("WGRAD_ROWS", 256):
        assert L.gr_wgrad_workspace_size(200000, 300, 200) > ws  # more splits, more slabs
        with pytest.raises(_lib.GrError, match="workspace"):
            _lib.call("gr_wgrad", fake, 300, None, fake, 200, fake, 128, 200000, 300, 200, fake,
                      None, fake, ws, None)
        desc = (ctypes.c_int64 * 18)(fake, 300, 0, fake, 200, 300, 200, fake, 0,
                                     fake, 300, 0, fake, 50, 300, 50, fake, fake)
        with pytest.raises(_lib.GrError, match="workspace"):
            _lib.call("gr_wgrad_multi", ctypes.addressof(desc), 2, fake, 128, 200000, 0, fake, ws,
                      None)
    with _lib.option("MIPS_SAMPLE_STRIDE", 64):
        ws_t = L.mips_topk_workspace_size(128, 10_000_000, 50, 200, 211)
    with _lib.option("MIPS_SAMPLE_STRIDE", 8):
        assert L.mips_topk_workspace_size(128, 10_000_000, 50, 200, 211) > ws_t
        with pytest.raises(_lib.GrError, match="workspace"):
            _lib.call("mips_topk", fake, fake, 10_000_000, 50, fake, 0, fake, 211, 128, 200, fake,
                      fake, fake, fake, ws_t, None)
    # the attention backward's dS tiles are optional: sized without them (ATTN_BWD_DS=0)
    # and launched with them on, it runs the recomputing form, which needs only the slabs
    # (tests/test_gpu_attention.py checks that form's results)
    with _lib.option("ATTN_BWD_DS", 0):
        slabs_only = L.hstu_attn_bwd_workspace_size(128, 211, 200, 1, 128)
    assert slabs_only < L.hstu_attn_bwd_workspace_size(128, 211, 200, 1, 128)


def test_launch_options_are_explicit_not_environment():
    """Launch options go through gr_set_option; the library reads no environment."""
    opts = _lib.parse_options()
    assert set(opts) == {"MIPS_FILTER_FP32", "MIPS_FILTER_WGS", "MIPS_FILTER_ROUNDS",
                         "MIPS_FORCE_FALLBACK", "ATTN_BWD_SPLIT", "ROWWAVE", "ATTN_BWD_PAIRS",
                         "ATTN_BWD_DS", "DETERMINISTIC", "WGRAD_ROWS", "PANEL_VEC",
                         "ATTN_BWD_WIDE_DS", "ATTN_BWD_WIDE_SPLIT", "MIPS_FILTER_PAIRED",
                         "MIPS_SAMPLE_STRIDE", "WGRAD_STREAM", "BOUNDARY_FUSE"}
    defaults = {"ROWWAVE": 1, "ATTN_BWD_PAIRS": 1, "PANEL_VEC": 1, "ATTN_BWD_DS": 1,
                "ATTN_BWD_WIDE_DS": 1, "ATTN_BWD_WIDE_SPLIT": 0, "MIPS_FILTER_PAIRED": 1,
                "WGRAD_STREAM": 1, "BOUNDARY_FUSE": 1}
    for n in opts:
        assert _lib.get_option(n) == defaults.get(n, 0), n
    with _lib.option("ATTN_BWD_SPLIT", 1):
        assert _lib.get_option("ATTN_BWD_SPLIT") == 1
    assert _lib.get_option("ATTN_BWD_SPLIT") == 0
    L = _lib.lib()
    assert L.gr_get_option(0) == -1 and L.gr_get_option(99) == -1
    assert L.gr_set_option(99, 1) != 0 and "unknown option" in L.gr_last_error().decode()
    with pytest.raises(_lib.GrError):
        _lib.set_option("MIPS_FILTER_WGS", 17)
    with pytest.raises(_lib.GrError):
        _lib.set_option("ROWWAVE", -1)
    # none of the library's own sources reads the environment (rocPRIM, linked for the
    # deterministic mode's radix sort, reads its own ROCPRIM_USE_ATOMIC_BLOCK_ID)
    csrc = os.path.join(os.path.dirname(_lib.LIB_PATH), "csrc")
    for f in sorted(os.listdir(csrc)):
        if f.endswith((".hip", ".cpp", ".h")):
            assert "getenv" not in open(os.path.join(csrc, f)).read(), f


def test_library_is_gfx950_code_object():
    """The fat binary embeds a gfx950 (MI355X) code object and nothing else."""
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    for other in (b"gfx942", b"gfx90a", b"sm_"):
        assert b"amdgcn-amd-amdhsa--" + other not in data
    assert ctypes.sizeof(ctypes.c_void_p) == 8


@pytest.mark.parametrize("struct", ["GrBoundaryBwd", "GrBoundaryFwd"])
def test_boundary_struct_layout_matches_header(tmp_path, struct):
    """ops.GrBoundaryBwd / GrBoundaryFwd (ctypes) have the C layout of include/gr_hstu.h's
    structs: same size and field offsets, checked against gcc on the header itself."""
    from mygenerativerecommenders_amd import ops
    GrBoundaryBwd = getattr(ops, struct)
    names = [f[0] for f in GrBoundaryBwd._fields_]
    src = tmp_path / "layout.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "gr_hstu.h"\nint main(void) {\n'
                   '  printf("%zu\\n", sizeof(' + struct + '));\n'
                   + "".join(f'  printf("%zu\\n", offsetof({struct}, {n}));\n' for n in names)
                   + "  return 0;\n}\n")
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.dirname(_lib.HEADER_PATH), str(src), "-o", str(exe)])
    got = [int(v) for v in subprocess.check_output([str(exe)], text=True).split()]
    assert got[0] == ctypes.sizeof(GrBoundaryBwd)
    assert got[1:] == [getattr(GrBoundaryBwd, n).offset for n in names]


def test_thread_options_are_per_thread():
    """gr_set_thread_option overrides an option for the calling thread only,
    so two threads that size and launch under different options never see each other's
    values (ctypes drops the GIL inside each call, so the threads really overlap in the
    library).  Each thread checks its workspace sizes against the values its options
    give when run alone, and a launch sized under the other thread's options is rejected
    (the check runs before any device work: fake pointers are never dereferenced)."""
    import threading
    L = _lib.lib()
    fake = 1 << 20
    # reference sizes, computed serially with process-wide options
    want = {}
    for rows, stride in ((4096, 64), (256, 8)):
        with _lib.option("WGRAD_ROWS", rows), _lib.option("MIPS_SAMPLE_STRIDE", stride):
            want[rows] = (L.gr_wgrad_workspace_size(200000, 300, 200),
                          L.mips_topk_workspace_size(128, 10_000_000, 50, 200, 211))
    assert want[256][0] > want[4096][0] and want[256][1] > want[4096][1]
    start = threading.Barrier(2)
    errors = []

    def worker(rows, stride, other_rows):
        try:
            _lib.set_thread_option("WGRAD_ROWS", rows)
            _lib.set_thread_option("MIPS_SAMPLE_STRIDE", stride)
            assert _lib.get_option("WGRAD_ROWS") == rows
            start.wait()
            for _ in range(2000):
                got = (L.gr_wgrad_workspace_size(200000, 300, 200),
                       L.mips_topk_workspace_size(128, 10_000_000, 50, 200, 211))
                assert got == want[rows], (rows, got, want[rows])
            if rows == 256:  # the other thread's (smaller) workspace is refused here
                with pytest.raises(_lib.GrError, match="workspace"):
                    _lib.call("gr_wgrad", fake, 300, None, fake, 200, fake, 128, 200000, 300, 200,
                              fake, None, fake, want[other_rows][0], None)
            _lib.clear_thread_option()
            assert _lib.get_option("WGRAD_ROWS") == 0  # back to the process-wide default
        except BaseException as e:  # noqa: BLE001 — reported by the main thread
            errors.append(e)

    ts = [threading.Thread(target=worker, args=(4096, 64, 256)),
          threading.Thread(target=worker, args=(256, 8, 4096))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors
    # the main thread never saw either override
    assert _lib.get_option("WGRAD_ROWS") == 0 and _lib.get_option("MIPS_SAMPLE_STRIDE") == 0
    with pytest.raises(_lib.GrError):
        _lib.set_thread_option("MIPS_FILTER_WGS", 17)
    assert L.gr_clear_thread_option(99) != 0
