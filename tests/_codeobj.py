"""Helpers for CPU tests that read the gfx950 code objects inside libgr_hstu.so.

The shared library's `.hip_fatbin` section holds one clang offload bundle per translation
unit.  `code_objects()` splits them, unbundles the gfx950 ELF of each with
clang-offload-bundler, and caches the results (keyed by the library's size and mtime);
`kernel_metadata()` reads the AMDGPU metadata notes (scratch, VGPR and spill counts);
`disassemble()` lists one kernel's instructions with their addresses and branch targets.
Only ROCm's own LLVM tools are used (no GPU)."""
from __future__ import annotations

import hashlib
import os
import re
import subprocess
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _tool(name):
    return os.path.join(LLVM, name)


def tools_present() -> bool:
    return all(os.path.exists(_tool(t)) for t in ("llvm-objcopy", "clang-offload-bundler",
                                                  "llvm-objdump", "llvm-readelf"))


def code_objects(lib_path: str) -> list[str]:
    st = os.stat(lib_path)
    key = hashlib.sha1(f"{os.path.abspath(lib_path)}:{st.st_size}:{st.st_mtime_ns}".encode()).hexdigest()[:16]
    d = os.path.join(tempfile.gettempdir(), f"gr_codeobj_{key}")
    done = os.path.join(d, "done")
    if os.path.exists(done):
        return [os.path.join(d, f) for f in sorted(os.listdir(d)) if f.endswith(".co")]
    os.makedirs(d, exist_ok=True)
    fat = os.path.join(d, "fat.bin")
    subprocess.check_call([_tool("llvm-objcopy"), "--dump-section", f".hip_fatbin={fat}", lib_path,
                           os.path.join(d, "stripped.so")])
    data = open(fat, "rb").read()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)] + [len(data)]
    out = []
    for n, (a, b) in enumerate(zip(starts, starts[1:])):
        part = os.path.join(d, f"b{n:02d}.bin")
        with open(part, "wb") as f:
            f.write(data[a:b])
        co = os.path.join(d, f"k{n:02d}.co")
        subprocess.check_call([_tool("clang-offload-bundler"), "--unbundle", "--type=o",
                               f"--targets={TARGET}", f"--input={part}", f"--output={co}"])
        out.append(co)
    open(done, "w").close()
    return out


def kernel_metadata(lib_path: str) -> dict:
    """{kernel symbol: {private_segment_fixed_size, vgpr_count, vgpr_spill_count,
    sgpr_spill_count, agpr_count}} over every code object."""
    meta = {}
    for co in code_objects(lib_path):
        notes = subprocess.check_output([_tool("llvm-readelf"), "--notes", co], text=True)
        for ent in re.split(r"\n\s+- \.agpr_count", notes)[1:]:
            ent = ".agpr_count" + ent

            def g(k):
                m = re.search(r"\." + k + r":\s+(\d+)", ent)
                return int(m.group(1)) if m else 0
            name = re.search(r"\.name:\s+(\S+)", ent).group(1)
            meta[name] = {k: g(k) for k in ("private_segment_fixed_size", "vgpr_count",
                                            "vgpr_spill_count", "sgpr_spill_count", "agpr_count")}
    return meta


def find_symbols(lib_path: str, pattern: str) -> dict:
    """{symbol: code object} for FUNC symbols matching the regex."""
    found = {}
    for co in code_objects(lib_path):
        syms = subprocess.check_output([_tool("llvm-readelf"), "-sW", co], text=True)
        for line in syms.splitlines():
            parts = line.split()
            if len(parts) >= 8 and parts[3] == "FUNC" and re.search(pattern, parts[7]):
                found[parts[7]] = co
    return found


_LINE = re.compile(r"^\s+(\S+)(.*?)\s*//\s*([0-9A-Fa-f]+):")
_TGT = re.compile(r"<(\S+?)\+0x([0-9a-fA-F]+)>")


def disassemble(co: str, symbol: str) -> list[tuple[int, str, str, int | None]]:
    """[(address, mnemonic, operands, branch target address or None)] of one function."""
    txt = subprocess.check_output([_tool("llvm-objdump"), "-d", "--no-show-raw-insn",
                                   f"--disassemble-symbols={symbol}", co], text=True)
    base = None
    syms = subprocess.check_output([_tool("llvm-readelf"), "-sW", co], text=True)
    for line in syms.splitlines():
        parts = line.split()
        if len(parts) >= 8 and parts[7] == symbol:
            base = int(parts[1], 16)
    assert base is not None, symbol
    return parse_listing(txt, symbol, base)


def parse_listing(txt: str, symbol: str, base: int) -> list[tuple[int, str, str, int | None]]:
    out = []
    for line in txt.splitlines():
        m = _LINE.match(line)
        if not m:
            continue
        mnem, ops, addr = m.group(1), m.group(2).strip(), int(m.group(3), 16)
        tgt = None
        t = _TGT.search(line)
        if t and t.group(1) == symbol and mnem.startswith(("s_cbranch", "s_branch")):
            tgt = base + int(t.group(2), 16)
        out.append((addr, mnem, ops, tgt))
    return out


VMEM_PREFIXES = ("global_", "buffer_", "flat_", "scratch_")


def check_dma_ring(instrs, ops: int) -> list[str]:
    """The hand-counted LDS-DMA ring of hstu_attn_bf16w.hip (v_from_p_ring_body and the dQ
    pass's ring): each loop waits `s_waitcnt vmcnt(ops)` then `s_barrier`, so between two
    such waits the only vector-memory instructions may be the `ops` inline-asm
    global_load_lds_dwordx4 of the next chunk.  Returns a list of violations (empty = OK)."""
    problems = []
    heads = [i for i, (_, mn, op, _) in enumerate(instrs)
             if mn == "s_waitcnt" and op == f"vmcnt({ops})" and i + 1 < len(instrs)
             and instrs[i + 1][1] == "s_barrier"]
    if not heads:
        return [f"no ring head (s_waitcnt vmcnt({ops}) + s_barrier) found"]
    for h in heads:
        haddr = instrs[h][0]
        back = [j for j in range(h + 1, len(instrs))
                if instrs[j][3] is not None and instrs[j][3] <= haddr]
        if not back:
            problems.append(f"ring head at {haddr:#x}: no backward branch closes the loop")
            continue
        j = back[0]
        lo = instrs[j][3]
        body = [x for x in instrs if lo <= x[0] <= instrs[j][0]]
        vmem = [x for x in body if x[1].startswith(VMEM_PREFIXES)]
        other = [x for x in vmem if x[1] != "global_load_lds_dwordx4"]
        for x in other:
            problems.append(f"loop {lo:#x}-{instrs[j][0]:#x}: compiler-issued {x[1]} {x[2]} at "
                            f"{x[0]:#x} shares the hand-counted vmcnt({ops})")
        dma = len(vmem) - len(other)
        if dma != ops:
            problems.append(f"loop {lo:#x}-{instrs[j][0]:#x}: {dma} LDS-DMA instructions per "
                            f"chunk, the wait counts {ops}")
    return problems
