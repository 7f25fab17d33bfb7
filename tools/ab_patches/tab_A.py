# A/B variant A: fine-bucket tables of 3072 slots, 512-lane workgroups, 4 keys per lane
s = open("group_hash.hip").read()
open("group_hash.hip", "w").write("#define SD_MIN_THREADS 512\n#define SD_MIN_TABLE 3072\n#define SD_MIN_ITEMS 4\n" + s)
