"""The committed per-config schedules (radiancecascade2dglobalillumination_amd/tuning/*.json) are well formed:
one variant and one order code per cascade level, variants the storage's kernels build (rc2dgi_rc_*.hip),
order codes of rc_logical_order's form, knobs the library knows (rc2dgi_set_tuning)."""
import glob
import json
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TUNING = os.path.join(ROOT, "radiancecascade2dglobalillumination_amd", "tuning")
CSRC = os.path.join(ROOT, "radiancecascade2dglobalillumination_amd", "csrc")


def variant_count():
    src = open(os.path.join(CSRC, "rc2dgi_kernels.hip")).read()
    body = src[src.index("kRcVariantNames[] = {"):]
    return len(re.findall(r'"[^"]+"', body[:body.index("};")]))


def built_variants(storage):
    """The rc_variant ids a storage's dispatcher launches as themselves (not as its default kernel)."""
    if storage == "f32":
        return set(range(variant_count()))
    src = open(os.path.join(CSRC, {"f16": "rc2dgi_rc_f16.hip", "rgba8": "rc2dgi_rc_u8.hip"}[storage])).read()
    return {0, 25} | {int(v) for v in re.findall(r"case (\d+):", src)}  # (25: k_rc_top, every storage)


KNOBS = {"rc_pal", "rc_skip", "rc_tail", "rc_wgproof", "jfa_lds", "jfa_coset", "shade_fused", "blur_path", "rc_chain", "jfa_rt", "shade_split", "side_overlap"}

FILES = sorted(glob.glob(os.path.join(TUNING, "*.json")))


def test_there_are_committed_schedules():
    assert len(FILES) >= 6


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(p) for p in FILES])
def test_schedule_file_is_well_formed(path):
    m = re.match(r"(\d+)x(\d+)_N(\d+)_rr([\d.]+)_(f32|f16|rgba8)\.json$", os.path.basename(path))
    assert m, "file name: WxH_N<n>_rr<range>_<storage>.json"
    W, H, N, storage = int(m.group(1)), int(m.group(2)), int(m.group(3)), m.group(5)
    d = json.load(open(path))
    assert d["config"].startswith(f"{W}x{H} N={N} ") and d["config"].endswith(storage)
    entries = [d] + list(d.get("strips", {}).values())
    for e in entries:
        assert len(e["rc_variant"]) == N and len(e["rc_order"]) == N
        for v in e["rc_variant"]:
            assert v in built_variants(storage), f"variant {v} is not built for {storage}"
        for code in e["rc_order"]:
            # px | py << 8 | dg << 16 | mode << 24 (0 patches, 1 oriented, 2 bands) | lc << 26 (XCD interleave)
            px, py, dg, mode, lc = code & 0xFF, (code >> 8) & 0xFF, (code >> 16) & 0xFF, (code >> 24) & 3, code >> 26
            base = code & ((1 << 26) - 1)
            assert 0 <= lc <= 31 and (base == 0 or (px > 0 and py > 0 and dg > 0 and mode in (0, 1, 2))), f"order code {code}"
    for k in d.get("knobs", {}):
        assert k in KNOBS or re.match(r"rc_(tail|mp|noproof|order|variant)_L\d+$", k), f"knob {k}"
