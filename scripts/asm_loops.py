"""Prints the basic-block structure of one kernel in a hipcc -S listing: each block's
label, instruction count, MFMA / VMEM / VALU / wait counts and its branch, so a hot
loop's per-iteration instruction mix can be read at a glance.
python scripts/asm_loops.py file.s kernel_symbol"""
import re
import sys


def main(path, name):
    s = open(path).read()
    a = s.index(name + ":")
    b = s.index(".Lfunc_end", a)
    blocks, cur = [], None
    for line in s[a:b].splitlines():
        t = line.strip()
        if re.match(r"^\.LBB\S+:", t) or t == name + ":":
            cur = {"label": t, "n": 0, "mfma": 0, "vmem": 0, "valu": 0, "wait": 0, "salu": 0,
                   "lds": 0, "br": ""}
            blocks.append(cur)
            continue
        if not t or t.startswith((";", ".")) or cur is None:
            continue
        op = t.split()[0]
        cur["n"] += 1
        if "mfma" in op:
            cur["mfma"] += 1
        elif op.startswith(("global_load", "buffer_load", "global_store", "buffer_store",
                            "global_atomic")):
            cur["vmem"] += 1
        elif op.startswith("ds_"):
            cur["lds"] += 1
        elif op.startswith("s_waitcnt"):
            cur["wait"] += 1
        elif op.startswith("v_"):
            cur["valu"] += 1
        elif op.startswith("s_"):
            cur["salu"] += 1
        if op.startswith(("s_cbranch", "s_branch")):
            cur["br"] = t
    for blk in blocks:
        print(f"{blk['label']:28s} n={blk['n']:4d} mfma={blk['mfma']:3d} vmem={blk['vmem']:3d} "
              f"valu={blk['valu']:4d} salu={blk['salu']:3d} lds={blk['lds']:3d} "
              f"wait={blk['wait']:3d}  {blk['br']}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
