# A/B variant: group_hash.hip with SD_SCATTER_BLKOFF=0
s = open("group_hash.hip").read()
open("group_hash.hip", "w").write("#define SD_SCATTER_BLKOFF 0\n" + s)
