# diagnosis: bucket_min returns right after its loads (launch + loads only)
s=open('group_hash.hip').read()
a="    __syncthreads();  // table initialised (first trip) / overflow flag visible\n    if (overflow) break;"
assert a in s; s=s.replace(a,"    __syncthreads();  // table initialised (first trip) / overflow flag visible\n    if (k[0] == 0x123456789ull && p[1] == 7u && v[2] == 9u) out[0] = 1;\n    return;\n    if (overflow) break;")
open('group_hash.hip','w').write(s)
