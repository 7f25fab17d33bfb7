# A/B variant: no region chain above 1.44M keys (totals + scatter + refine + tables)
s = open("group_hash.hip").read()
open("group_hash.hip", "w").write("#define SD_BIG_REGIONS 0\n" + s)
