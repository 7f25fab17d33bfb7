# A/B variant: group_hash.hip with SD_RESERVE_OVERLAP=0 (wait for each trip's reservation before the scan)
s = open("group_hash.hip").read()
open("group_hash.hip", "w").write("#define SD_RESERVE_OVERLAP 0\n" + s)
