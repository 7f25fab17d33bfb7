# A/B variant C: fine-bucket tables of 6144 slots, 1024-lane workgroups, 2 keys per lane
s = open("group_hash.hip").read()
open("group_hash.hip", "w").write("#define SD_MIN_THREADS 1024\n#define SD_MIN_TABLE 6144\n#define SD_MIN_ITEMS 2\n" + s)
