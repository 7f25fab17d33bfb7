# A/B variant: every lane of every staged trip stores (the coarse scatter too)
s = open("group_hash.hip").read()
a = "    if (!RESERVE || t0 < trip_n) {"
assert s.count(a) == 1
s = s.replace(a, "    if (true) {")
open("group_hash.hip", "w").write(s)
