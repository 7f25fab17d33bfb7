# A/B variant: the fine tables' Object count on one device counter
s = open("group_hash.hip").read()
open("group_hash.hip", "w").write("#define SD_GROUP_OBJ_SHARDS 1\n" + s)
