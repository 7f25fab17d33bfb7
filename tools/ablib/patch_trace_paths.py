# diagnosis: per-phase wall times of sd_cas_generate_cas_ids_from_paths on stderr
s=open('sd_hip_cas.cpp').read()
s=s.replace('#include "ctx_internal.h"', '#include "ctx_internal.h"\n#include <chrono>\nstatic double now_us() { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count(); }',1)
a="""  for (size_t w = 0; w < nw && rc == 0; w++) {
    const int b = (int)(w & 1);
    if (w >= 2 && (rc = finish(w - 2))) break;  // slot b free again
    gather(w, pin0 + b * slot);
    const size_t f0 = w * GATHER_WINDOW, m = std::min(GATHER_WINDOW, n - f0);
    rc = enqueue_staged(c, plans[w], sizes + f0, m, pin0 + b * slot, dev0 + b * slot, done[b]);
  }
  for (size_t w = nw >= 2 ? nw - 2 : 0; w < nw && rc == 0; w++) rc = finish(w);"""
b="""  double tg = 0, te = 0, tf = 0, t0 = now_us();
  for (size_t w = 0; w < nw && rc == 0; w++) {
    const int b = (int)(w & 1);
    if (w >= 2 && (rc = finish(w - 2))) break;  // slot b free again
    double a0 = now_us();
    gather(w, pin0 + b * slot);
    double a1 = now_us();
    const size_t f0 = w * GATHER_WINDOW, m = std::min(GATHER_WINDOW, n - f0);
    rc = enqueue_staged(c, plans[w], sizes + f0, m, pin0 + b * slot, dev0 + b * slot, done[b]);
    double a2 = now_us();
    tg += a1 - a0; te += a2 - a1;
  }
  double a3 = now_us();
  for (size_t w = nw >= 2 ? nw - 2 : 0; w < nw && rc == 0; w++) rc = finish(w);
  tf = now_us() - a3;
  fprintf(stderr, "TRACE n=%zu setup=%.1f gather=%.1f enqueue=%.1f finish=%.1f total=%.1f\\n", n, t0 - tstart, tg, te, tf, now_us() - tstart);"""
assert a in s; s=s.replace(a,b)
a="""  HIP_TRY(c, hipSetDevice(c->device));
  // Content length per file: sampled 57,344; whole file = its actual length (cas.rs:29"""
b="""  double tstart = now_us();
  HIP_TRY(c, hipSetDevice(c->device));
  // Content length per file: sampled 57,344; whole file = its actual length (cas.rs:29"""
assert a in s; s=s.replace(a,b)
open('sd_hip_cas.cpp','w').write(s)
