# A/B variant: group_hash.hip with SD_COARSE_BITS=9 (2^9 coarse buckets above 1.44 M keys)
s = open("group_hash.hip").read()
open("group_hash.hip", "w").write("#define SD_COARSE_BITS 9\n" + s)
