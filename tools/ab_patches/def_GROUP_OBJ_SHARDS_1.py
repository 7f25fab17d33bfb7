# A/B variant: group_hash.hip with SD_GROUP_OBJ_SHARDS=1
s = open("group_hash.hip").read()
open("group_hash.hip", "w").write("#define SD_GROUP_OBJ_SHARDS 1\n" + s)
