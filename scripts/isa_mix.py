#!/usr/bin/env python3
"""Instruction mix of the k_rc_level kernels the committed bench schedule runs.

Compiles the RC translation units to gfx950 assembly with -DRC2DGI_ISA_SECTIONS (section markers
in rc2dgi_rc.h: setup / march / tail / stage_write / merge), splits each kernel at the markers and
counts the instructions of every section by class:

  valu      plain 32-bit VALU (2 cycles per wave64 instruction on a SIMD-32 with >= 2 waves,
            MI355X_MICROARCH.md "Wave scheduling" / constants table)
  valu_pk   v_pk_*_f32 (twice the lanes of work: 4 cycles; the f32 VALU peak is 64 FLOP/clk/SIMD
            whether packed or not, cdna_hip_programming.md §MFMA rate)
  valu_tr   transcendentals v_rcp/v_rsq/v_sqrt/v_exp/v_log/v_sin/v_cos (8 vs 4 cycles for one
            wave alone in the constants table: twice a plain op, 4 cycles)
  valu_64   64-bit VALU (v_*_b64 / v_*_u64 / f64; priced 4 cycles -- an assumption, not measured)
  salu, smem, vmem, lds, wait, branch

Usage: scripts/isa_mix.py [--json out.json]   (no GPU needed; hipcc only)
"""
import argparse
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
CSRC = os.path.join(ROOT, "radiancecascade2dglobalillumination_amd", "csrc")
TUS = ["rc2dgi_rc_f32a.hip", "rc2dgi_rc_f32b.hip"]
COST = {"valu": 2, "valu_pk": 4, "valu_tr": 4, "valu_64": 4}
TRANS = ("v_rcp", "v_rsq", "v_sqrt", "v_exp", "v_log", "v_sin", "v_cos")


def classify(op):
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith(("s_load", "s_buffer_load", "s_store", "s_dcache")):
        return "smem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith(("s_branch", "s_cbranch", "s_setpc", "s_endpgm")):
        return "branch"
    if op.startswith(("s_nop", "s_barrier", "s_setprio", "s_sleep")):
        return "other"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        base = op.split("_e32")[0].split("_e64")[0].split("_sdwa")[0].split("_dpp")[0]
        if base.startswith("v_pk_") and base.endswith("_f32"):
            return "valu_pk"
        if base.startswith(TRANS):
            return "valu_tr"
        if re.search(r"_(b64|u64|i64|f64)$", base) or base in ("v_lshl_add_u64",):
            return "valu_64"
        return "valu"
    return "other"


def kernels(asm_text):
    """{mangled kernel name: [lines]} of every k_rc_level instantiation."""
    out, cur, name = {}, None, None
    for line in asm_text.split("\n"):
        m = re.match(r"^(_ZN6rc2dgi10k_rc_level\S*):", line)
        if m:
            name, cur = m.group(1), []
            continue
        if cur is not None:
            if line.strip().startswith(".Lfunc_end"):
                out[name] = cur
                cur = None
            else:
                cur.append(line)
    return out


def template_args(name):
    """(TX, TY, PY, PD, TOP, P2S, UNR, DL, GI, Z0) from the mangled name."""
    m = re.search(r"k_rc_levelILi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELb([01])ELb([01])ELi(\d+)ELi(\d+)ENS_(\d+)(\w+?)ELb([01])E",
                  name)
    if not m:
        return None
    g = m.groups()
    return dict(TX=int(g[0]), TY=int(g[1]), PY=int(g[2]), PD=int(g[3]), TOP=g[4] == "1", P2S=g[5] == "1",
                UNR=int(g[6]), DL=int(g[7]), GI=g[9][:int(g[8])], Z0=g[10] == "1")


def sections(lines):
    sec = "setup"
    counts = collections.defaultdict(collections.Counter)
    for line in lines:
        if ";@section" in line:
            sec = line.split(";@section")[1].strip()
            continue
        t = line.strip()
        if not t or t.startswith((";", ".", "//")) or t.endswith(":"):
            continue
        op = t.split()[0]
        counts[sec][classify(op)] += 1
    return counts


def compile_asm(tu, sections_on, tmp):
    from radiancecascade2dglobalillumination_amd import _build

    out = os.path.join(tmp, tu + (".sec" if sections_on else "") + ".s")
    cmd = [_build.hipcc()] + _build.FLAGS + ["-I", os.path.join(ROOT, "include"), "--offload-device-only", "-S",
                                             os.path.join(CSRC, tu), "-o", out]
    if sections_on:
        cmd.insert(1, "-DRC2DGI_ISA_SECTIONS")
    subprocess.run([c for c in cmd if c != "-fPIC"], check=True, capture_output=True)
    with open(out) as f:
        return f.read()


VARIANT_SHAPE = {0: (16, 16, 1, 1, 1, 0), 6: (32, 8, 2, 1, 1, 0), 13: (16, 16, 1, 1, 32, 0),
                 18: (16, 16, 1, 1, 1, 2), 19: (16, 16, 1, 1, 1, 3), 2: (16, 16, 2, 1, 1, 0)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json")
    ap.add_argument("--schedule", default=os.path.join(ROOT, "radiancecascade2dglobalillumination_amd", "tuning",
                                                       "4096x4096_N6_rr2_f32.json"))
    a = ap.parse_args()
    with open(a.schedule) as f:
        sched = json.load(f)
    N = len(sched["rc_variant"])
    with tempfile.TemporaryDirectory() as tmp:
        sec_k, prod_k = {}, {}
        for tu in TUS:
            sec_k.update(kernels(compile_asm(tu, True, tmp)))
            prod_k.update(kernels(compile_asm(tu, False, tmp)))
    # keyed on the configuration and the per-level variants it was built for: bench.py prices a run's VALU
    # instructions with this mix only when its own (config, rc_variant) match
    m = re.match(r"(\d+)x(\d+) N=(\d+)", sched.get("config", ""))
    cfg = f"{m.group(1)}x{m.group(2)}_N{m.group(3)}" if m else None
    rep = {"key": {"config": cfg, "rc_variant": [int(v) for v in sched["rc_variant"]]},
           "schedule": os.path.relpath(a.schedule, ROOT), "cost_cycles": COST, "levels": {}}
    for L in range(N):
        v = sched["rc_variant"][L]
        TX, TY, PY, PD, UNR, DL = VARIANT_SHAPE[v]
        want = dict(TX=TX, TY=TY, PY=PY, PD=PD, TOP=L == N - 1, P2S=True, UNR=UNR, DL=DL, GI="GiF32",
                    Z0=(L == 0 and L != N - 1))
        names = [n for n in sec_k if template_args(n) == want]
        pn = [n for n in prod_k if template_args(n) == want]
        if not names or not pn:
            print(f"L{L}: kernel for variant {v} not found", file=sys.stderr)
            continue
        sc = sections(sec_k[names[0]])
        prod = sections(prod_k[pn[0]])
        tot_prod = collections.Counter()
        for c in prod.values():
            tot_prod.update(c)
        row = {"variant": v, "shape": f"{TX}x{TY}x{PY} DL{DL} UNR{UNR}",
               "sections": {s: dict(c) for s, c in sc.items()}, "product_total": dict(tot_prod)}
        valu = {k: tot_prod.get(k, 0) for k in COST}
        nv = sum(valu.values())
        row["valu_static"] = nv
        row["valu_cycles_per_inst"] = round(sum(valu[k] * COST[k] for k in COST) / max(nv, 1), 3)
        rep["levels"][f"L{L}"] = row
        print(f"L{L} v{v} {row['shape']}: product VALU {nv} (pk {valu['valu_pk']}, tr {valu['valu_tr']}, "
              f"64b {valu['valu_64']}), SALU {tot_prod.get('salu', 0)}, VMEM {tot_prod.get('vmem', 0)}, "
              f"LDS {tot_prod.get('lds', 0)}; mean VALU cost {row['valu_cycles_per_inst']} cyc")
        for s in ("setup", "march", "tail", "stage_write", "merge"):
            c = sc.get(s, {})
            if c:
                print(f"    {s:12s} valu {c.get('valu', 0):4d} pk {c.get('valu_pk', 0):3d} tr {c.get('valu_tr', 0):3d} "
                      f"64b {c.get('valu_64', 0):3d} salu {c.get('salu', 0):4d} vmem {c.get('vmem', 0):3d} "
                      f"lds {c.get('lds', 0):3d} wait {c.get('wait', 0):3d}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rep, f, indent=1)


if __name__ == "__main__":
    main()
