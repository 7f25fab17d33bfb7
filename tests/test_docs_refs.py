"""DESIGN.md's evidence references resolve: every `profiles/...` path it cites (globs
included) exists in the tree, and every `tools/...` script it cites exists or is marked as
kept in git history."""
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_design_references_exist():
    s = open(os.path.join(ROOT, "DESIGN.md")).read()
    missing = []
    for r in sorted(set(re.findall(r"`(profiles/[^`\s]+)`", s))):
        p = os.path.join(ROOT, r)
        if not (glob.glob(p) if "*" in r else os.path.exists(p.rstrip("/"))):
            missing.append(r)
    for m in re.finditer(r"`(tools/[^`\s]+)`(, in git history)?", s):
        if not m.group(2) and not os.path.exists(os.path.join(ROOT, m.group(1))):
            missing.append(m.group(1))
    assert not missing, missing
