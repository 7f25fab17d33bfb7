# timing-only ablation: bucket tables without the duplicates' scattered out[] stores
s = open("group_hash.hip").read()
a = "          if (mv != v[j]) out[p[j]] = mv;  // out[] was prefilled with the own value\n"
assert s.count(a) == 1
s = s.replace(a, "          if (mv == 0xFFFFFFFFu) out[p[j]] = mv;\n")
open("group_hash.hip", "w").write(s)
