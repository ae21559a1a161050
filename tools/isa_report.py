#!/usr/bin/env python3
"""ISA report of the product kernels from the gfx950 assembly (`make -C zig-raytracing-weekend_amd/csrc isa`).

For each kernel whose symbol contains one of the given substrings: register and scratch use as the
compiler reports them (.num_vgpr, ScratchSize, Occupancy), the instruction histogram by class, and
every loop (a backward branch to an earlier label) with its static instruction counts -- the walk
loop is the one that loads BVH nodes (ds_read_b128 from the LDS stage, or global_load_dwordx4).

Usage: python tools/isa_report.py build/isa/rtw_wavefront_all.s wf_step_cldsILj0E wf_traceILj0ELb0E wf_tail_cldsILj0E
       [--json out.json]
       python tools/isa_report.py build/isa/rtw_wavefront_all.s --resources profiles/isa_resources.json
         the build-stamped resource table of every wavefront kernel (VGPR / SGPR / scratch / occupancy / code
         bytes), stamped with the in-tree library's rtw_build_id() (tests/test_abi.py checks the stamp);
         `make -C zig-raytracing-weekend_amd/csrc resources` runs both steps
"""
from __future__ import annotations

import argparse
import collections
import json
import re
import sys

CLASSES = [
    ("v_pk_fp32", re.compile(r"^v_pk_(fma|mul|add|mov)_(f32|b32)")),
    ("v_pk_other", re.compile(r"^v_pk_")),
    ("v_fma_mix", re.compile(r"^v_fma_mix")),
    ("v_fma", re.compile(r"^v_(fma|fmac|fmaak|fmamk)_f32")),
    ("v_mul_f32", re.compile(r"^v_mul_f32")),
    ("v_add_sub_f32", re.compile(r"^v_(add|sub|subrev)_f32")),
    ("v_minmax_f32", re.compile(r"^v_(min|max|min3|max3|med3|minimum|maximum)\w*_f32")),
    ("v_cmp", re.compile(r"^v_cmpx?_")),
    ("v_cndmask", re.compile(r"^v_cndmask")),
    ("v_transcendental", re.compile(r"^v_(rcp|rsq|sqrt|exp|log|sin|cos)_")),
    ("v_div_helpers", re.compile(r"^v_div_")),
    ("v_mov", re.compile(r"^v_(mov|readfirstlane|readlane|writelane)")),
    ("v_int", re.compile(r"^v_(and|or|xor|lshl|lshr|ashr|add_u|add_co|addc|sub_u|sub_co|subb|mul_lo|mul_hi|mad_u|"
                         r"bfe|bfi|perm|alignbit|cvt|bcnt|mbcnt|ffbh|ffbl|not|add3|lshl_add|lshl_or|and_or|or3|xad|"
                         r"mad_i|mad_u64|min_u|max_u|min_i|max_i)")),
    ("v_other", re.compile(r"^v_")),
    ("ds", re.compile(r"^ds_")),
    ("global_load", re.compile(r"^(global|buffer|flat)_load")),
    ("global_store", re.compile(r"^(global|buffer|flat)_store")),
    ("global_atomic", re.compile(r"^(global|buffer|flat)_atomic")),
    ("s_waitcnt", re.compile(r"^s_waitcnt")),
    ("s_branch", re.compile(r"^s_(cbranch|branch)")),
    ("salu", re.compile(r"^s_")),
]


def classify(m):
    for name, rx in CLASSES:
        if rx.match(m):
            return name
    return "other"


def kernels(text):
    """(symbol, body lines, meta dict) for every kernel function of the file."""
    out = []
    for m in re.finditer(r"^(_Z\S+):\s*; @", text, re.M):
        sym = m.group(1)
        end = text.find(".Lfunc_end", m.end())
        body = text[m.end():end].splitlines()
        meta = {}
        for key, rx in (("vgpr", rf"\.set {re.escape(sym)}\.num_vgpr, (\d+)"),
                        ("agpr", rf"\.set {re.escape(sym)}\.num_agpr, (\d+)"),
                        ("sgpr", rf"\.set {re.escape(sym)}\.numbered_sgpr, (\d+)"),
                        ("private_seg", rf"\.set {re.escape(sym)}\.private_seg_size, (\d+)")):
            mm = re.search(rx, text)
            if mm:
                meta[key] = int(mm.group(1))
        tail = text[end:end + 4000]
        for key, rx in (("scratch", r"; ScratchSize: (\d+)"), ("occupancy", r"; Occupancy: (\d+)"),
                        ("lds_static", r"; LDSByteSize: (\d+)"), ("code_bytes", r"; codeLenInByte = (\d+)")):
            mm = re.search(rx, tail)
            if mm:
                meta[key] = int(mm.group(1))
        out.append((sym, body, meta))
    return out


def instrs(lines):
    """(index, mnemonic, line) of the instructions, and label -> index of the next instruction."""
    ins, labels = [], {}
    for ln in lines:
        s = ln.strip()
        if not s or s.startswith(";") or s.startswith("."):
            if re.match(r"^\.LBB\w+:", s):
                labels[s.split(":")[0]] = len(ins)
            continue
        mn = s.split()[0]
        if mn.endswith(":"):
            continue
        ins.append((len(ins), mn, s))
    return ins, labels


def loops(ins, labels):
    """Backward branches: (head, tail) instruction index ranges, innermost first."""
    out = []
    for i, mn, s in ins:
        if mn.startswith("s_cbranch") or mn == "s_branch":
            tgt = s.split()[-1]
            if tgt in labels and labels[tgt] <= i:
                out.append((labels[tgt], i))
    return sorted(set(out), key=lambda r: r[1] - r[0])


def hist(seq):
    c = collections.Counter(classify(mn) for _, mn, _ in seq)
    return dict(sorted(c.items(), key=lambda kv: -kv[1]))


def demangle(sym):
    """_ZN12_GLOBAL__N_113wf_step_clds2ILj0ELj768EEEv... -> wf_step_clds2<0u, 768u> (template ints / bools only)."""
    pre = "_ZN12_GLOBAL__N_1"
    if not sym.startswith(pre):
        return sym
    m = re.match(r"(\d+)", sym[len(pre):])
    if not m:
        return sym
    n = int(m.group(1))
    k = len(pre) + len(m.group(1))
    name, rest = sym[k:k + n], sym[k + n:]
    if not rest.startswith("I"):
        return name
    args = re.findall(r"L([jib])(\d+)E", rest[:rest.index("EE") + 1] if "EE" in rest else rest)
    pretty = [("true" if v == "1" else "false") if t == "b" else (v + "u" if t == "j" else v) for t, v in args]
    return f"{name}<{', '.join(pretty)}>"


def write_resources(text, path):
    import ctypes
    import os
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = ctypes.CDLL(os.path.join(repo, "zig-raytracing-weekend_amd", "librtw_gpu.so"))
    lib.rtw_build_id.restype = ctypes.c_char_p
    table = {}
    for sym, body, meta in kernels(text):
        table[demangle(sym)] = {k: meta.get(k) for k in ("vgpr", "agpr", "sgpr", "scratch", "occupancy", "code_bytes")}
    out = {"build_id": lib.rtw_build_id().decode(), "source": "tools/isa_report.py --resources over "
           "`make isa` (both wavefront translation units, product flags)", "kernels": table}
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    spill = {k: v["scratch"] for k, v in table.items() if v.get("scratch")}
    print(f"{len(table)} kernels, build {out['build_id']}; with scratch: {spill}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("names", nargs="*")
    ap.add_argument("--json")
    ap.add_argument("--resources", help="write the build-stamped resource table of every kernel to this file")
    a = ap.parse_args()
    text = open(a.asm).read()
    if a.resources:
        write_resources(text, a.resources)
        return
    report = {}
    for sym, body, meta in kernels(text):
        if not any(n in sym for n in a.names):
            continue
        ins, labels = instrs(body)
        lp = []
        for h, t in loops(ins, labels):
            seg = ins[h:t + 1]
            mns = [mn for _, mn, _ in seg]
            walk = any(m.startswith("ds_read_b128") or m.startswith("global_load_dwordx4") for m in mns) and any(
                m.startswith("v_fma_mix") for m in mns)
            lp.append({"first": h, "last": t, "instructions": len(seg), "walk": walk,
                       "valu": sum(1 for m in mns if m.startswith("v_")), "salu": sum(1 for m in mns if m.startswith("s_")),
                       "classes": hist(seg)})
        report[sym] = {"meta": meta, "instructions": len(ins), "classes": hist(ins), "loops": lp}
        print(f"== {sym}")
        print(f"   {meta}  static instructions {len(ins)}")
        print("   classes:", ", ".join(f"{k} {v}" for k, v in hist(ins).items()))
        for l in lp:
            if l["walk"] or l["instructions"] >= 40:
                tag = "WALK " if l["walk"] else ""
                print(f"   {tag}loop [{l['first']}..{l['last']}] {l['instructions']} instr "
                      f"(VALU {l['valu']}, SALU {l['salu']}): " + ", ".join(f"{k} {v}" for k, v in l["classes"].items()))
    if a.json:
        json.dump(report, open(a.json, "w"), indent=1)
    if not report:
        print("no kernel matched", a.names, file=sys.stderr)
        sys.exit(1)


if __name__ == "__main__":
    main()
