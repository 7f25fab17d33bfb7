# A/B variant: no small-batch region chain (totals + scatter + big tables for every batch)
s = open("group_hash.hip").read()
open("group_hash.hip", "w").write("#define SD_SMALL_REGIONS 0\n" + s)
