# A/B variant: group_hash.hip with 2^8 coarse buckets at every size (SD_COARSE10_KEYS huge)
s = open("group_hash.hip").read()
open("group_hash.hip", "w").write("#define SD_COARSE10_KEYS 0xFFFFFFFFFFull\n" + s)
