#!/usr/bin/env python3
"""A/B patch for tools/build_variant.sh: set `#define NAME VALUE` (the `#ifndef NAME` default)
in every csrc file of the current directory that defines it.  Usage: patch_define.py NAME VALUE"""
import glob
import re
import sys

name, value = sys.argv[1], sys.argv[2]
hits = 0
for f in glob.glob("*.hip") + glob.glob("*.h") + glob.glob("*.hpp") + glob.glob("*.cpp"):
    s = open(f).read()
    t, k = re.subn(rf"(#define {re.escape(name)}) \S+", rf"\g<1> {value}", s)
    if k:
        open(f, "w").write(t)
        hits += k
if not hits:
    sys.exit(f"patch_define: no #define {name} found")
print(f"{name}={value} ({hits} site(s))")
