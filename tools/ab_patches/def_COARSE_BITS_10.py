# A/B variant: group_hash.hip with SD_COARSE_BITS=10 (2^10 coarse buckets above 1.44 M keys)
s = open("group_hash.hip").read()
open("group_hash.hip", "w").write("#define SD_COARSE_BITS 10\n" + s)
