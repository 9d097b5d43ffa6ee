"""CPU checks on the gfx950 machine code that ships in libgr_hstu.so (no GPU needed).

1. The inline-asm LDS-DMA rings.  The dV and dQ passes of
   the wide bf16 attention backward (hstu_attn_bf16w.hip: v_from_p_ring_body and the dQ
   ring) issue their LDS-DMA from inline asm, which hipcc does not count, and wait
   `s_waitcnt vmcnt(OPS)` with OPS = D32 / 2 + 2 their own pieces per chunk.  That wait is
   only right while the ring loop holds no other vector-memory instruction: a compiler
   change or an edit that moves one load or store into the loop would turn it into a
   silent race.  The test disassembles every ring instantiation and checks the loop.
   A second test feeds the checker a listing with one inserted load and expects it to fail.
2. Scratch and VGPR spills: every kernel's metadata is read; the fused
   attention + layer-boundary kernels and the DMA-ring kernels must use no scratch and
   spill nothing, and no kernel outside a short list of known, measured exceptions may
   start using scratch."""
import re

import pytest

from mygenerativerecommenders_amd import _lib
from tests import _codeobj as C

pytestmark = pytest.mark.skipif(not C.tools_present(), reason="ROCm LLVM tools not installed")

RING = r"_ZN2gr24attn_bwd_bf16w_(vp|dq)_kernelILi(\d+)E"


def _ring_kernels():
    found = C.find_symbols(_lib.LIB_PATH, RING)
    out = []
    for sym, co in sorted(found.items()):
        d32 = int(re.search(RING, sym).group(2))
        if d32 % 2 == 0:  # odd D32 takes the two-buffer builtin form (no asm ring)
            out.append((sym, co, d32 // 2 + 2))
    return out


def test_dma_ring_loops_hold_only_their_counted_dma():
    kernels = _ring_kernels()
    # the even instantiations of both passes (d = 192 and d = 256 heads at least)
    assert {re.search(RING, s).group(1) for s, _, _ in kernels} == {"vp", "dq"}
    assert len(kernels) >= 4, [s for s, _, _ in kernels]
    for sym, co, ops in kernels:
        instrs = C.disassemble(co, sym)
        problems = C.check_dma_ring(instrs, ops)
        assert not problems, (sym, problems)


def test_dma_ring_checker_catches_an_inserted_load():
    sym, co, ops = _ring_kernels()[0]
    instrs = C.disassemble(co, sym)
    assert not C.check_dma_ring(instrs, ops)
    # one compiler-issued load right after the ring's barrier (inside the loop)
    h = next(i for i, x in enumerate(instrs) if x[1] == "s_waitcnt" and x[2] == f"vmcnt({ops})"
             and instrs[i + 1][1] == "s_barrier")
    a = instrs[h + 1][0]
    bad = instrs[:h + 2] + [(a + 2, "global_load_dword", "v1, v[2:3], off", None)] + instrs[h + 2:]
    problems = C.check_dma_ring(bad, ops)
    assert any("global_load_dword" in p for p in problems), problems
    # one DMA piece fewer than the wait counts
    i = next(i for i, x in enumerate(instrs) if i > h and x[1] == "global_load_lds_dwordx4")
    short = instrs[:i] + instrs[i + 1:]
    assert any("LDS-DMA instructions per chunk" in p for p in C.check_dma_ring(short, ops))


# Kernels that use scratch today, each measured and not on the default path of any
# BASELINE config (values: allowed bytes of private segment).
SCRATCH_OK = {
    # narrow bf16 dQ at D32 = 8 (d in (96, 128] with the narrow bf16 form; the wide form,
    # hstu_attn_bf16w.hip, serves d > 128)
    "_ZN2gr23attn_bwd_bf16_dq_kernelILi8ELi8ELi32ELi8ELb1EE": 96,
    # row-wave gate_o at D = 256 with hdv = 64 (C3 widths take the row panel)
    "rowwave_kernelILi16ELi4ENS_7RwGateOILi16ELi4ELi2EEEEEvT1_": 108,
    # f32 ln_uvqk backward row panel at 8 column groups (a local array indexed per row)
    "rowpanel_kernelILi8ELi64ENS_*OpLnUvqkBwd": 20,
    # top-k merges: a small per-lane array indexed dynamically
    "_ZN2gr17mips_merge_kernelENS_9MergeArgsE": 16,
    "_ZN2gr24mips_filter_merge_kernelENS_15FilterMergeArgsE": 16,
    "mips_select_kernelILi64ELi1EEEvNS_10SelectArgsEi": 16,
    # rocPRIM's radix sort (deterministic-mode table gradient), not ours
    "rocprim": 80,
}


def _allowed(name):
    for k, v in SCRATCH_OK.items():
        if all(part in name for part in k.split("*")):
            return v
    return 0


def test_no_new_scratch_or_vgpr_spills():
    meta = C.kernel_metadata(_lib.LIB_PATH)
    assert len(meta) > 500
    over = {n: m for n, m in meta.items() if m["private_segment_fixed_size"] > _allowed(n)}
    assert not over, over
    # the fused attention + layer-boundary kernels (RwStage weight panels held in registers
    # beside the attention) and the DMA-ring kernels: no scratch, no VGPR spill
    fused = [n for n in meta if re.search(r"hstu_attn_fwd_bnd_kernel|attn_bwd_dq_bnd_kernel|"
                                          r"attn_bwd_bf16w_(vp|dq|k)_kernel|attn_fwd_bf16w_kernel", n)]
    assert len(fused) >= 10, fused
    for n in fused:
        m = meta[n]
        assert m["private_segment_fixed_size"] == 0 and m["vgpr_spill_count"] == 0, (n, m)
