"""CPU checks of the measurement tooling that builds from the product source.

tools/sweep/htime.py inserts the diagnostic timestamps of tools/hier_attrib.py into a generated
copy of flame_amd/csrc/fedagg.hip at fixed anchors; every anchor must match once, so a product
change that moves one is caught here (no sweep fork to drift).  The sweep tools' variants name
only FLAME_T_* knobs the product source defines.
"""
import importlib.util
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "flame_amd", "csrc", "fedagg.hip")


def _load(path, name):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_htime_anchors_apply_to_the_product_source(tmp_path):
    htime = _load(os.path.join(ROOT, "tools", "sweep", "htime.py"), "htime")
    out = htime.generate(str(tmp_path / "stamped.hip"))
    text = open(out).read()
    assert text.count("FLAME_HT(") >= 5 and "flame_sweep_htime" in text
    # only stamps were added: the product source minus the inserted lines is unchanged
    prod = open(SRC).read()
    assert len(text) > len(prod)


def test_sweep_variants_name_existing_knobs():
    knobs = set(re.findall(r"#ifndef (FLAME_T_\w+)", open(SRC).read()))
    assert {"FLAME_T_CLIENT_UNROLL", "FLAME_T_HBL", "FLAME_T_OPT_WGC"} <= knobs
    for tool in ("kernel_sweep.py", "hier_sweep.py"):
        src = open(os.path.join(ROOT, "tools", tool)).read()
        used = set(re.findall(r'"(FLAME_T_\w+)"', src))
        assert used and used <= knobs, (tool, used - knobs)
