# A/B variant: the small-batch region chain's cursors contiguous (8 cache lines)
s = open("group_hash.hip").read()
open("group_hash.hip", "w").write("#define SD_REGION_CURSOR_STRIDE 1\n" + s)
