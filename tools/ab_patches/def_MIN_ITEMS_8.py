# A/B variant: group_hash.hip with SD_MIN_ITEMS=8
s = open("group_hash.hip").read()
open("group_hash.hip", "w").write("#define SD_MIN_ITEMS 8\n" + s)
