# A/B variant: the fused chain on 2^9 regions (two 512-lane, 6,144-slot tables per CU)
s = open("sd_mix.h").read()
open("sd_mix.h", "w").write(s.replace("#define SD_REGION_BITS 8", "#define SD_REGION_BITS 9"))
