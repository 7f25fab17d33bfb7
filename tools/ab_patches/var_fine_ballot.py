# A/B variant: the fine tables also sum their fresh keys per wave (ballots)
s = open("group_hash.hip").read()
a = "    if (THREADS >= 1024) {\n      // the big tables"
assert s.count(a) == 1
s = s.replace(a, "    if (THREADS >= 512) {\n      // the big tables")
open("group_hash.hip", "w").write(s)
