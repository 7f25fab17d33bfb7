# A/B variant: group_hash.hip with 2^10 coarse buckets above 1.44 M keys (SD_COARSE10_KEYS 0)
s = open("group_hash.hip").read()
open("group_hash.hip", "w").write("#define SD_COARSE10_KEYS 0\n" + s)
