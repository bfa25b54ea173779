"""Every tracked file under profiles/ is evidence something cites (VERDICT r05 hygiene): a file
name (or a glob such as ``r05fin2_*``) in DESIGN.md, INTEGRATION.md, tools/README.md or
profiles/README.md, or a line of profiles/HISTORY_CITED.txt (files only round 4's DESIGN.md
appendices cite: ``git show 672be85:DESIGN.md``).  Uncited files are pruned, not kept."""
import fnmatch
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOCS = ("DESIGN.md", "INTEGRATION.md", "tools/README.md", "profiles/README.md")


def _tracked():
    try:
        out = subprocess.check_output(["git", "ls-files", "profiles"], cwd=ROOT, stderr=subprocess.DEVNULL)
    except (OSError, subprocess.CalledProcessError):
        pytest.skip("not a git checkout")
    return [f for f in out.decode().split() if f not in ("profiles/README.md", "profiles/HISTORY_CITED.txt")]


def _expand(p):
    """Brace groups ({FETCH,WRITE}_SIZE) -> one pattern per alternative, recursively."""
    m = re.search(r"\{([^{}]*)\}", p)
    if not m:
        return {p}
    out = set()
    for alt in m.group(1).split(","):
        out |= _expand(p[:m.start()] + alt + p[m.end():])
    return out


def _patterns():
    text = "".join(open(os.path.join(ROOT, d)).read() for d in DOCS)
    toks = set(re.findall(r"(?:[A-Za-z0-9_.*\-\[\]]|\{[^{}\s]*\})+", text))
    pats = set()
    for t in toks:
        if re.search(r"(r0\d|traffic|\.log|\.csv|\.json)", t):
            pats |= _expand(t)
    return pats


def test_every_profile_is_cited():
    pats = _patterns()
    hist = {ln.strip() for ln in open(os.path.join(ROOT, "profiles", "HISTORY_CITED.txt"))
            if ln.strip() and not ln.startswith("#")}
    uncited = [f for f in _tracked()
               if os.path.basename(f) not in hist
               and not any(fnmatch.fnmatch(os.path.basename(f), p) or fnmatch.fnmatch(f, p) for p in pats)]
    assert not uncited, f"{len(uncited)} profiles/ files cited nowhere (cite them or prune them): {uncited[:20]}"


def test_history_list_names_existing_files():
    hist = [ln.strip() for ln in open(os.path.join(ROOT, "profiles", "HISTORY_CITED.txt"))
            if ln.strip() and not ln.startswith("#")]
    missing = [h for h in hist if not os.path.exists(os.path.join(ROOT, "profiles", h))]
    assert not missing, missing[:20]
