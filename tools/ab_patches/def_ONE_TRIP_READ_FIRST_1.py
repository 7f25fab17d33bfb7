# A/B variant: one-trip buckets probe read-first (CAS only an empty slot)
s = open("group_hash.hip").read()
open("group_hash.hip", "w").write("#define SD_ONE_TRIP_READ_FIRST 1\n" + s)
