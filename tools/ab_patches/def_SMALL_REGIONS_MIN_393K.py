# A/B variant: the small-batch region chain only above 393,216 keys (the first cut)
s = open("group_hash.hip").read()
open("group_hash.hip", "w").write("#define SD_SMALL_REGIONS_MIN (256ull * 1536)\n" + s)
