#!/usr/bin/env python3
"""Randomised parity stress for the path gather (sd_cas_generate_cas_ids_from_paths and
sd_cas_file_metadata_from_paths: the pread pool, the streamed single-window pipeline with its
whole-files-first order, the windowed double-buffered one, the re-read of whole files whose
length changed): a pool of files on tmpfs (config 1's log-uniform 1 KiB..10 MiB sizes plus
edge sizes around 102,400 and 8 KiB multiples, empty files, a directory, missing paths) is
drawn from at random every iteration — batch sizes from 1 to 6,000 paths, repeats of one path
inside a batch, caller sizes that are right, stale (shrunk/grown metadata) or 0, or no sizes
at all, and random kernel shapes (default, four-files-per-wave K1L, lane-per-file) — and each
result is compared with the C oracle's gather + hash of the same (path, size) list
(oracle/cas_fast.c, orc_generate_cas_keys_paths: the cas.rs read/seek sequence).  With
--checksums every iteration also runs the validator over a random batch of the same pool
(sd_cas_file_checksums: hash.rs's full-content BLAKE3) against the oracle's digest of each
file's bytes.  Prints one JSON line per iteration and a summary; exit 1 on any mismatch."""
import argparse
import errno
import json
import os
import shutil
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=180)
    ap.add_argument("--files", type=int, default=3000)
    ap.add_argument("--seed", type=int, default=2027)
    ap.add_argument("--root", default="/dev/shm/sdcas_stress_paths")
    ap.add_argument("--checksums", action="store_true")
    a = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401  (loads the HIP runtime first, like the product's users)
    from spacedrive_amd import CasEngine
    from spacedrive_amd.cas import STATUS_NO_CAS
    from oracle.pyoracle import Oracle
    eng = CasEngine(0)
    orc = Oracle()
    rng = np.random.default_rng(a.seed)
    shutil.rmtree(a.root, ignore_errors=True)
    os.makedirs(a.root)
    try:
        paths, sizes = [], []
        edge = [0, 1, 63, 64, 1023, 1024, 1025, 8191, 8192, 16384, 16385, 102399, 102400, 102401,
                102402, 118784, 120000]
        for i in range(a.files):
            s = edge[i] if i < len(edge) else int(np.exp(rng.uniform(np.log(1024), np.log(10 << 20))))
            p = os.path.join(a.root, f"p{i:05d}")
            with open(p, "wb") as fh:
                fh.write(rng.integers(0, 256, s, dtype=np.uint8).tobytes())
            paths.append(p)
            sizes.append(s)
        os.mkdir(os.path.join(a.root, "adir"))
        paths += [os.path.join(a.root, "adir"), os.path.join(a.root, "missing")]
        sizes += [4096, 5000]
        sizes = np.array(sizes, dtype=np.uint64)
        pool = len(paths)
        t_end = time.time() + a.seconds
        it = fails = 0
        while time.time() < t_end:
            m = int(rng.choice([int(rng.integers(1, 17)), int(rng.integers(16, 200)),
                                int(rng.integers(200, 2100)), int(rng.integers(2000, 6000))],
                               p=[0.25, 0.4, 0.2, 0.15]))
            idx = rng.integers(0, pool, m)
            if m > 4 and rng.random() < 0.3:  # one path several times in the batch
                idx[rng.integers(0, m, max(1, m // 10))] = idx[0]
            bp = [paths[i] for i in idx]
            mode = ["given", "stale", "none"][it % 3]
            bs = sizes[idx].copy()
            if mode == "stale":  # metadata that no longer matches the file, and zeros
                k = rng.random(m)
                bs[k < 0.1] = (bs[k < 0.1] * rng.uniform(0.3, 3.0, int((k < 0.1).sum()))).astype(np.uint64)
                bs[(k >= 0.1) & (k < 0.13)] = 0
            shape = ["default", "seg16", "lane"][(it // 3) % 3]
            if shape == "seg16":
                eng.set_chunkpar_split(0, 0)
            elif shape == "lane":
                eng.set_latency_threshold(0, 0)
            try:
                if mode == "none":
                    keys, status, msz = eng.file_metadata_from_paths(bp)
                else:
                    keys, status = eng.generate_cas_keys_from_paths(bp, bs)
                    msz = bs
            finally:
                eng.set_latency_threshold()
                eng.set_chunkpar_split()
            # the oracle on the same (path, metadata size) list: rows the metadata decides
            # (stat errors, directories, length 0) have no cas read
            if mode == "none":
                want_sz = np.array([os.stat(p).st_size if os.path.exists(p) else 0 for p in bp],
                                   dtype=np.uint64)
                sz_ok = bool((msz[status >= 0] == want_sz[status >= 0]).all())
            else:
                want_sz, sz_ok = bs, True
            wk, ws = orc.generate_cas_keys_paths(bp, want_sz, 16, simd=True)
            # the batch oracle's whole-file buffer holds 100 KiB: a file that grew past it
            # under small metadata (cas.rs:29 reads the actual file) takes the one-path oracle
            for i in np.nonzero(ws == -errno.E2BIG)[0]:
                try:
                    wk[i], ws[i] = int(orc.generate_cas_id(bp[i], int(want_sz[i])), 16), 0
                except OSError as e:
                    wk[i], ws[i] = 0, -e.errno
            ok = sz_ok
            for i in range(m):
                p = bp[i]
                if mode != "none" and want_sz[i] == 0:  # a caller size of 0: no read at all
                    ok &= bool(status[i] == STATUS_NO_CAS and keys[i] == 0)
                elif os.path.isdir(p):
                    ok &= bool(status[i] == -errno.EISDIR and keys[i] == 0)
                elif not os.path.exists(p):
                    ok &= bool(status[i] == -errno.ENOENT and keys[i] == 0)
                elif want_sz[i] == 0:
                    ok &= bool(status[i] == STATUS_NO_CAS and keys[i] == 0)
                else:
                    ok &= bool(status[i] == ws[i] and (ws[i] != 0 or keys[i] == wk[i]))
                if not ok:
                    print(json.dumps({"it": it, "bad_row": i, "path": p, "size": int(want_sz[i]),
                                      "status": int(status[i]), "want_status": int(ws[i]),
                                      "key": f"{int(keys[i]):016x}", "want": f"{int(wk[i]):016x}"}),
                          flush=True)
                    break
            ck = None
            if a.checksums:
                cm = int(rng.integers(1, 400))
                cidx = rng.integers(0, pool, cm)
                cp = [paths[i] for i in cidx]
                dig, cerr = eng.file_checksums(cp)
                ck = True
                for p, d, e in zip(cp, dig, cerr):
                    if os.path.isdir(p):
                        ck &= bool(e == errno.EISDIR and d is None)
                    elif not os.path.exists(p):
                        ck &= bool(e == errno.ENOENT and d is None)
                    else:
                        with open(p, "rb") as fh:
                            ck &= bool(e == 0 and d == orc.blake3(fh.read()).hex())
                    if not ck:
                        print(json.dumps({"it": it, "bad_checksum": p, "errno": int(e), "digest": d}), flush=True)
                        break
                ok &= ck
            fails += 0 if ok else 1
            print(json.dumps({"it": it, "n": m, "mode": mode, "shape": shape, "checksums": ck,
                              "errors": int((status < 0).sum()), "no_cas": int((status == STATUS_NO_CAS).sum()),
                              "ok": ok}), flush=True)
            it += 1
        print(json.dumps({"iterations": it, "failures": fails, "seconds": a.seconds}), flush=True)
    finally:
        shutil.rmtree(a.root, ignore_errors=True)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
