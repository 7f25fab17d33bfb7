# A/B variant: one sd_bucket_min workgroup per fine bucket (no resident streaming grid)
s = open("group_hash.hip").read()
open("group_hash.hip", "w").write("#define SD_MIN_STREAM 0\n" + s)
