# 256-thread bucket_min workgroups (one 2,048-key trip)
s=open('group_hash.hip').read()
a="constexpr int MIN_THREADS = 512;"
assert a in s; s=s.replace(a,"constexpr int MIN_THREADS = 256;")
open('group_hash.hip','w').write(s)
