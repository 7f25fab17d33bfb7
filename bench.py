#!/usr/bin/env python3
"""Benchmark: cas_ids/s + hashed GB/s (whole node) on MI355X — BASELINE.json's metric.

Workload (one "step"): every rank hashes its resident batch of sampled-path files
(BASELINE configs 3/4: 57,344 gathered bytes per file, 57,352-B BLAKE3 message, 30 %
duplicate content) with K1 and groups the cas keys into Objects — locally on one GPU,
by key-range all-to-all over RCCL on several.  Inputs are synthesized on the device
before the timed region (data: synthetic) and are resident in HBM when it starts.
Weak scaling: FILES_PER_GPU (default 1,310,720 = 20 x 65,536, the MI355X file-per-lane
quantum; 75.2 GB/GPU) per rank per step, so one step at 8 GPUs is the 10M-file headline
job (10.49 M files).  Steps are pipelined the way a production job
would run them: step i's grouping (incl. its RCCL exchange, issued from a worker thread
so its host syncs never delay the next K1) runs on a side stream while steps i+1 and i+2
are hashed (keys triple-buffered); every step's hash AND grouping complete inside the
timed region (--no-overlap serialises them).

Output: ONE JSON line on rank 0 (driver contract), with
  roofline      — K1 (sd_cas_sampled_kernel; K1G at N=1), timed by HIP events on its own
                  stream, priced as SURVEY.md §8(d) prices it: 953 compressions x 792 spec
                  int32 ops per file / kernel time vs the guide's int32 VALU peak (256 CUs x 4
                  SIMDs x 32 lanes x 2.4 GHz = 78.6 T lane-ops/s); secondary views: the HBM
                  byte view (vs 8 TB/s) and PMC traffic, and from ONE committed gpurun session
                  (profiles/r05_valu_power.json, marked measured_in_this_run=false) the
                  counter-based VALU instruction rate and VALU busy, the compute-only ceiling
                  of K1's instruction stream per shader cycle and the power-capped clock;
                  plus rocm-smi power / sclk sampled live during this run's sustained steps;
  sustained     — the same steps back to back for ~--sustain-seconds after the timed region
                  (the DVFS-settled rate, long enough for an outside utilisation sampler);
  e2e           — BASELINE config 3 as worded: sampled files streamed from pinned host
                  memory (a pinned ring reused cyclically, every file copied H2D over PCIe)
                  through K1, PCIe-inclusive; never `value` (rank 0, N=1);
  cpu_baseline  — the oracle's AVX-512 16-lane CPU path (oracle/cas_fast.c) on a bounded
                  sample of the SAME files on the host cores (rank 0 at every N, the other
                  ranks at a barrier; threads: cpu_threads); the sample's keys are also
                  checked against the GPU's.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MSG_BYTES = 57352            # le64(size) || 57,344 sampled bytes
COMPRESSIONS = 953           # 897 chunk blocks + 56 parents per sampled message
SPEC_OPS = 792               # int32 ops per compression (7 rounds x 8 G x 14 + 8)
HW_OPS = 680                 # VALU instructions per compression as compiled (add3/alignbit)
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: 8.0 TB/s spec
# grouping (group_hash.hip): see group_bytes_per_key (the minima of duplicates are the only
# other stores)
def group_bytes_per_key(n: int) -> int:
    """Algorithmic HBM bytes per key of the standalone grouping: up to 1.44 M
    keys the region chain (read key 8, prefill rep 4, region row 12, tables read it 12); up to
    40 M the two-level region chain (+ the refine: count pass 8, rows 12/12); above, the
    partition chain (totals 8 + prefill 4 + scatter 8/12 + count 8 + refine 12/12 + read 12)."""
    if n <= 256 * 5632:
        return 36
    return 68 if n <= 40_000_000 else 76


FUSED_REGION_BITS = 8  # sd_mix.h REGION_BITS
FUSED_MAX_FILES = 256 * 5632  # the fused chain's single-level regions (sd_cas_hash_group_sampled_dev)


def eng_region_capacity(n: int) -> int:
    """Rows per coarse-bucket region of the fused chain (group_hash.hip region_capacity)."""
    regions = 1 << FUSED_REGION_BITS
    mean = n / regions
    var = mean * (1 - 1 / regions)
    sd = 1
    while sd * sd < var:
        sd += 1
    return int(mean) + 1 + 8 * sd + 64
VALU_PEAK_TOPS = 256 * 128 * 2.4e9 / 1e12  # 256 CUs x 4 SIMD32 x 32 lanes x 2.4 GHz = 78.6
PCIE_PEAK_GBS = 64.0         # PCIe Gen5 x16 per direction


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--files-per-gpu", type=int, default=1_310_720,
                    help="20 x 65,536 (the MI355X file-per-lane quantum): 10.49 M files per step at 8 GPUs")
    ap.add_argument("--dup-permille", type=int, default=300)
    ap.add_argument("--seed", type=int, default=0x5DCA50004)
    ap.add_argument("--cpu-seconds", type=float, default=6.0)
    ap.add_argument("--sustain-seconds", type=float, default=10.0,
                    help="back-to-back steps after the timed region (0 = skip)")
    ap.add_argument("--e2e-files", type=int, default=10_485_760,
                    help="files streamed from pinned host memory for the e2e sub-object (0 = skip)")
    ap.add_argument("--e2e-ring", type=int, default=131_072,
                    help="pinned host ring (files) the e2e stream cycles through, divided over "
                         "the ranks (>= 16,384 files = 0.94 GB per rank, far beyond any host "
                         "cache): the node's pinned total stays 7.5 GB at any n_gpus")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-overlap", dest="overlap", action="store_false",
                    help="group step i before hashing step i+1 (default: overlap them)")
    ap.add_argument("--exchange", action="store_true",
                    help="use the key-range all-to-all grouping even at N=1 (RCCL world 1): "
                         "measures the exchange path's cost on one GPU")
    ap.add_argument("--inline-group", action="store_true",
                    help="issue the grouping from the main thread (A/B of the worker thread)")
    ap.add_argument("--unfused", action="store_true",
                    help="N=1: K1 + the standalone grouping chain on the side stream (the round-2 "
                         "pipeline) instead of K1G (K1 partitioning its own keys) + bucket tables")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    rehearsal = bool(os.environ.get("SD_BENCH_ONE_DEVICE"))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `python bench.py --gpus N`: launch the N ranks ourselves, before any GPU call here
        sys.exit(spawn_ranks(args.gpus, rehearsal))

    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        fail(f"bench: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    if rehearsal:
        # rehearsal of the N > 1 code path with every rank on one GPU (RCCL refuses two
        # ranks on one device, so the exchange goes through gloo): not a measurement
        local = 0
    elif torch.cuda.device_count() < world:
        fail(f"bench: {world} ranks need {world} visible GPUs, found {torch.cuda.device_count()} "
             "(SD_BENCH_ONE_DEVICE=1 rehearses the N > 1 path on one GPU)")
    torch.cuda.set_device(local)
    sharded = world > 1 or args.exchange
    if world == 1 and args.exchange:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if sharded:
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        if dist.get_world_size() != args.gpus:
            fail(f"bench: the process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")

    from spacedrive_amd import CasEngine
    from spacedrive_amd.shard import (HipShardOps, exchange_bytes_per_step, fixed_capacity,
                                      sharded_group)

    eng = CasEngine(local)
    F = args.files_per_gpu
    file0 = rank * F
    dev = torch.device("cuda", local)
    content = torch.empty((F, 57344), dtype=torch.uint8, device=dev)
    sizes = torch.empty(F, dtype=torch.int64, device=dev)
    # keys triple-buffered: step i's grouping (side stream) overlaps steps i+1 and i+2's
    # hashing, so a grouping that waits for CU slots behind K1 never stalls the next K1
    NBUF = 3
    keys = [torch.empty(F, dtype=torch.int64, device=dev) for _ in range(NBUF)]
    rep = torch.empty(F, dtype=torch.int32, device=dev)
    # N=1: the fused chain — K1G partitions its own keys into fixed-capacity coarse-bucket
    # regions (two sets, alternating), the bucket tables of step i run on the side stream
    # while step i+1 hashes; each step's rep in its own buffer
    fused = (not sharded and not args.unfused and F % eng.batch_quantum == 0
             and F <= FUSED_MAX_FILES)
    reps = [torch.empty(F, dtype=torch.int32, device=dev) for _ in range(NBUF)] if fused else None
    ovf = torch.zeros(1, dtype=torch.int32, device=dev)
    eng.synth_sampled(args.seed, file0, F, content, sizes, 57344, dup_permille=args.dup_permille)
    torch.cuda.synchronize()
    ops = HipShardOps(eng)
    main = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    hashed = [torch.cuda.Event() for _ in range(NBUF)]
    grouped = [torch.cuda.Event() for _ in range(NBUF)]
    pending = [None] * NBUF
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    results = []      # the last step's ShardResult (sharded runs)
    overflows = []    # per-step overflow flags of the fixed-capacity exchange (device)
    resolve_in_step = [False]  # read each step's flag inside the step (after an overflow)
    # fixed per-peer capacity: the exchange needs no host sync (spacedrive_amd/shard.py)
    capacity = fixed_capacity(F, world) if sharded else None
    # The exchange path reads part sizes back to the host (all_to_all_single needs host
    # split lists), so it blocks its caller: it runs on a worker thread, and the main
    # thread only ever waits on it when it reuses that step's key buffer.
    worker = None
    if not args.inline_group:
        worker = ThreadPoolExecutor(1, initializer=torch.cuda.set_device, initargs=(local,))

    def group(i: int):
        """Object grouping of step i's keys on the side stream (RCCL exchange when sharded)."""
        b = i % NBUF
        with torch.cuda.stream(side):
            side.wait_event(hashed[b])
            if fused:
                eng.group_regions(F, reps[b], stream=side.cuda_stream, want_objects=False)
            elif not sharded:
                eng.group(keys[b], rep, want_objects=False)  # K4h + K5h, async
            else:
                r = sharded_group(keys[b], file0, ops, capacity=capacity)
                if r.overflow is not None:
                    if resolve_in_step[0]:
                        # the fallback mode: an overflowed fixed-capacity part is redone with
                        # the exact exchange inside the step (collective, on this worker
                        # thread; the flag read is one host sync per step)
                        overflows.append(int(r.overflow.item()))
                        r.resolve()
                    else:
                        # the flag stays on the device; it is read once after the timed loop
                        overflows.append(r.overflow.clone())
                results[:] = [r]
            grouped[b].record(side)

    def launch_group(i: int):
        b = i % NBUF
        # the fused chain's tables must be enqueued before the next batch's hash_regions
        # (they group the context's LAST batch): from the main thread; no host sync in them
        pending[b] = worker.submit(group, i) if worker is not None and not fused else group(i)

    def wait_group(b: int):
        if pending[b] is not None:
            if worker is not None and not fused:
                pending[b].result()
            main.wait_event(grouped[b])
            pending[b] = None

    def run(n: int, timed: bool):
        for i in range(n):
            b = i % NBUF
            wait_group(b)                       # keys[b] free again
            if timed:
                ev[i][0].record(main)
            if fused:  # K1G on the main stream
                eng.hash_regions_sampled(content, sizes, keys[b], reps[b], ovf)
            else:
                eng.hash_sampled(content, sizes, keys[b])      # K1 on the main stream
            if timed:
                ev[i][1].record(main)
            hashed[b].record(main)
            launch_group(i)
            if not args.overlap:
                wait_group(b)
        for b in range(NBUF):
            wait_group(b)

    def timed_region() -> float:
        results.clear()
        overflows.clear()
        ovf.zero_()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(args.steps, True)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    run(args.warmup, False)
    torch.cuda.synchronize()
    dt = timed_region()
    # world 1 (--exchange) runs the exact form: its part sizes are read on the host per step
    host_syncs_per_step = 1 if sharded and world == 1 else 0
    if sharded and overflows and not resolve_in_step[0]:
        # the fixed-capacity flags of the timed steps, read after the loop (no host sync
        # inside a step); any overflow means that step's rep needed the exact redo, so the
        # timed region is run again with the in-step redo (one flag read per step)
        fl = torch.stack([f.reshape(()) for f in overflows]).max().reshape(1).to(torch.int64)
        dist.all_reduce(fl, op=dist.ReduceOp.MAX)
        if int(fl.item()):
            resolve_in_step[0] = True
            host_syncs_per_step = 1
            dt = timed_region()
    last_keys = keys[(args.steps - 1) % NBUF]
    res = results[-1] if results else None
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    # every rank's K1 mean (slot r = rank r; a summed vector, so gloo rehearsals work too)
    km = torch.zeros(world, dtype=torch.float64, device=dev)
    km[rank] = kern_ms
    if sharded:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(km)
    dt = float(t.item())
    k1_ms_ranks = km.cpu().tolist()
    kern_ms = max(k1_ms_ranks)

    # objects (for the record) — outside the timed region
    fused_rec = None
    if not sharded:
        objects = eng.group(last_keys, rep)
    if fused:
        # every timed step's regions must have held their keys (else the step's rep would
        # need the standalone regroup); the last step's rep == the standalone grouping's
        timed_overflow = int(ovf.item())
        ovf.zero_()
        last_rep = reps[(args.steps - 1) % NBUF]
        rep_parity = bool(torch.equal(last_rep, rep))
        # the bucket tables alone, serially after K1G (inside the steps they share the CUs
        # with the next K1G on the side stream): HIP events on the stream they run on
        tabs = []
        for _ in range(3):
            a_, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            eng.hash_regions_sampled(content, sizes, last_keys, last_rep, ovf)
            a_.record(main)
            eng.group_regions(F, last_rep, want_objects=False)
            b_.record(main)
            b_.synchronize()
            tabs.append(a_.elapsed_time(b_))
        ovf.zero_()
        fobj = eng.hash_group_sampled(content, sizes, last_keys, last_rep, ovf)
        fobj_rep_parity = bool(torch.equal(last_rep, rep))
        fused_rec = {"tables_ms": float(np.median(tabs)), "tables_ms_all": tabs,
                     "objects": fobj,
                     "parity_vs_standalone": rep_parity and fobj_rep_parity and fobj == objects,
                     # an overflowed region is regrouped by its table workgroup inside the step
                     # (exact, on the device): the flag counts the slower path, never a wrong rep
                     "timed_steps_overflowed": timed_overflow,
                     "region_capacity": eng_region_capacity(F),
                     "note": "K1G (sd_cas_sampled_group_kernel: K1 + the coarse-bucket partition "
                             "of its own keys into fixed-capacity regions) + ONE bucket-table "
                             "launch (sd_bucket_min_regions); tables_ms = that launch alone, "
                             "after K1G, HIP events on its stream"}
    if sharded:
        # timed steps whose fixed-capacity exchange overflowed (redone exactly inside the step
        # in the fallback mode; 0 in the sync-free mode, else the run was repeated)
        n_overflow = sum(int(f.item()) if torch.is_tensor(f) else f for f in overflows)
        objects = res.objects
    # the grouping alone (after the timed region: inside the steps it overlaps the next K1
    # on a side stream and shares the CUs with it, so its own speed is measured serially)
    group_ms = group_ms_sync = group12_ms = group12_objects = lsd12 = None
    if not sharded:
        # (a) each call synchronised: includes the host's enqueue latency of its 2-4 launches
        # (the GPU idles ~4 us between the first two: profiles/r02b_group_chain_trace.txt);
        # (b) 10 calls back to back: the GPU time per grouping as the pipelined steps see it,
        # where the chain is enqueued ahead behind the hashing
        gts = []
        for _ in range(5):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(main)
            eng.group(last_keys, rep, want_objects=False)
            b.record(main)
            b.synchronize()
            gts.append(a.elapsed_time(b))
        group_ms_sync = float(np.median(gts))
        gb = []
        for _ in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(main)
            for _ in range(10):
                eng.group(last_keys, rep, want_objects=False)
            b.record(main)
            b.synchronize()
            gb.append(a.elapsed_time(b) / 10)
        group_ms = float(np.median(gb))
        # the same grouping at one rank's share of config 4 (12.5 M keys, 30 % duplicates,
        # two partition levels: 76 B/key), random keys generated on the device
        g = torch.Generator(device=dev)
        g.manual_seed(args.seed)
        nk, nd = 12_500_000, 3_750_000
        base = torch.randint(-2 ** 63, 2 ** 63 - 1, (nk - nd,), dtype=torch.int64, device=dev, generator=g)
        big = torch.cat([base, base[torch.randint(0, nk - nd, (nd,), device=dev, generator=g)]])
        big = big[torch.randperm(nk, device=dev, generator=g)]
        rep_big = torch.empty(nk, dtype=torch.int32, device=dev)
        eng.group(big, rep_big, want_objects=False)
        gb = []
        for _ in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(main)
            for _ in range(5):
                eng.group(big, rep_big, want_objects=False)
            b.record(main)
            b.synchronize()
            gb.append(a.elapsed_time(b) / 5)
        group12_ms = float(np.median(gb))
        group12_objects = eng.group(big, rep_big)
        lsd12 = lsd_sort_leg(eng, big, rep_big, group12_objects, main)
        del big, base, rep_big

    # the N > 1 exchange alone (partition + fixed-capacity all-to-all + grouping of the
    # received keys + mirror all-to-all), serially after the timed region, max over ranks
    exchange_ms = None
    exchange_phases = None
    if sharded:
        xs, phases = [], []
        for _ in range(3):
            dist.barrier()
            torch.cuda.synchronize()
            marks = [("start", torch.cuda.Event(enable_timing=True))]
            marks[0][1].record()

            def mark(name: str) -> None:
                e = torch.cuda.Event(enable_timing=True)
                e.record()
                marks.append((name, e))
            t1 = time.perf_counter()
            sharded_group(last_keys, file0, ops, capacity=capacity, mark=mark)
            torch.cuda.synchronize()
            xs.append(time.perf_counter() - t1)
            phases.append([marks[j - 1][1].elapsed_time(marks[j][1]) for j in range(1, len(marks))])
        names = [m[0] for m in marks[1:]]
        ph = torch.tensor(np.median(np.array(phases), axis=0), dtype=torch.float64, device=dev)
        xt = torch.tensor([float(np.median(xs)) * 1e3], dtype=torch.float64, device=dev)
        dist.all_reduce(xt, op=dist.ReduceOp.MAX)
        dist.all_reduce(ph, op=dist.ReduceOp.MAX)
        exchange_ms = float(xt.item())
        exchange_phases = dict(zip(names, ph.cpu().tolist()))

    # sustained: the same pipelined steps back to back (DVFS-settled; long enough for an
    # outside utilisation sampler to see the GPU busy), after the headline timed region
    sustained = None
    smi_live = None
    if args.sustain_seconds > 0:
        n_sus = max(1, int(args.sustain_seconds / (dt / args.steps)))
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        smi = SmiSampler(torch.cuda.get_device_properties(local)) if rank == 0 else None
        t0 = time.perf_counter()
        run(n_sus, False)
        torch.cuda.synchronize()
        if smi is not None:
            smi_live = smi.stop()
        ts = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        if sharded:
            dist.all_reduce(ts, op=dist.ReduceOp.MAX)
        sus_dt = float(ts.item())
        sustained = {"steps": n_sus, "seconds": sus_dt, "value": world * F * n_sus / sus_dt,
                     "n_gpus": world,
                     "unit": "cas_ids/s", "ms_per_step": sus_dt / n_sus * 1e3}

    e2e = None
    if args.e2e_files > 0:
        e2e = e2e_leg(eng, content, sizes, last_keys, args, world, rank, dev,
                      dist if sharded else None)

    files_total = world * F * args.steps
    value = files_total / dt
    gbs = files_total * MSG_BYTES / dt / 1e9
    achieved = F * MSG_BYTES / (kern_ms / 1e3) / 1e9  # per-GPU kernel GB/s
    valu = F * COMPRESSIONS * SPEC_OPS / (kern_ms / 1e3) / 1e12
    valu_hw = F * COMPRESSIONS * HW_OPS / (kern_ms / 1e3) / 1e12

    # HBM bytes per launch from PMC (TCC_MISS_sum x 128-B lines, committed summary of the
    # separate rocprofv3 --pmc pass on the same kernel), scaled to this launch's files
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_sampled_group_kernel.json" if fused
                       else "pmc_sampled_kernel.json")
    if os.path.exists(pmc):
        with open(pmc) as fh:
            per_file = json.load(fh).get("hbm_bytes_per_file")
            if per_file is not None:
                traffic = per_file * F

    # VALU evidence of the headline kernel and the power-capped clock: the counters come from
    # ONE committed gpurun session (tools/gpu_r5_valu_power.sh -> profiles/r05_valu_power.json:
    # rocprofv3 --pmc pass, compute-only K1 ceiling and rocm-smi probe on the same box); the
    # live part (power + sclk while the sustained steps run) is measured by this run
    valu_busy, power = valu_power_evidence("sd_cas_sampled_group_kernel" if fused else "sd_cas_sampled_kernel",
                                           F, kern_ms, sustained, smi_live)

    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu = cpu_baseline(content, sizes, last_keys, args.cpu_seconds)
        if world > 1:
            cpu["ranks_idle_meanwhile"] = world - 1
    if world > 1:
        dist.barrier()

    n_gpus = dist.get_world_size() if sharded else 1
    if rank == 0:
        line = {
            "metric": "cas_ids/sec + hashed GB/s (whole node), 10M files at 1/2/4/8 MI355X",
            "value": value,
            "unit": "cas_ids/s",
            "hashed_gb_per_s": gbs,
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (value / cpu["value"]) if cpu else None,
            "vs_baseline_basis": ("value / cpu_baseline.value: BASELINE.json's north_star names the "
                                  "reference CPU path on the same box's host cores as THE baseline "
                                  "(BASELINE.md publishes no number for this metric)"),
            "dtype": "u32",
            "data": "synthetic (on-device splitmix64 content, 30% duplicates), resident in HBM",
            "config": {
                "workload": "sampled-path cas_id (57,352-B BLAKE3 message/file) + Object grouping; "
                            f"{F} files/GPU/step ({world * F} per step at n_gpus={world})",
                "files_per_gpu": F,
                "dup_permille": args.dup_permille,
                "parallelism": f"shard-by-file x{world}" + (" + RCCL key-range all-to-all" if sharded else ""),
                "pipeline": (("K1G (K1 + partition of its keys into fixed-capacity bucket "
                              "regions) on the main stream; step i's bucket tables on a side "
                              "stream overlap step i+1's K1G" if fused else
                              "grouping of step i on a side stream (issued from a worker thread) "
                              "overlaps hashing of steps i+1 and i+2") if args.overlap
                             else "hash then group, serial"),
                "grouping": "fused" if fused else ("exchange" if sharded else "standalone chain"),
                "objects": objects,
                "exchange": None if not sharded else {
                    "backend": dist.get_backend(), "world_size": dist.get_world_size(),
                    "rehearsal_one_device": rehearsal,
                    "capacity_per_peer": capacity[0], "spill_per_peer": capacity[1],
                    "bytes_sent_per_rank_per_step": exchange_bytes_per_step(world, capacity),
                    "bytes_sent_per_step_all_ranks": world * exchange_bytes_per_step(world, capacity),
                    "host_syncs_per_step": host_syncs_per_step,
                    "host_syncs_note": ("0: every step's fixed-capacity overflow flag stays on the "
                                        "device and is read once after the timed loop; 1: an "
                                        "overflow was seen, so the steps were re-timed with the "
                                        "flag read (and the exact redo) inside each step"),
                    "timed_steps_overflowed": n_overflow,
                    "serial_ms": exchange_ms,
                    "serial_ms_phases": exchange_phases,
                    "serial_ms_note": "one step's exchange + grouping alone (max over ranks, "
                                      "after the timed region; phases = HIP events on the "
                                      "issuing stream between the phase boundaries, median of "
                                      "3, max over ranks); inside the steps it overlaps "
                                      "the next K1 on a side stream"},
            },
            "roofline": {
                # achieved = files x 953 compressions x 792 spec int32 ops /
                # K1 time, vs the guide's int32 VALU peak (78.6 T lane-ops/s).  BLAKE3 is
                # integer ARX with no contraction (no MFMA path) and K1 moves ~0.4 of HBM
                # peak, so VALU is the binding roof.
                "kernel": "sd_cas_sampled_group_kernel" if fused else "sd_cas_sampled_kernel",
                "bound": "valu",
                "bound_note": ("BLAKE3 is 32-bit integer ARX with no contraction: no MFMA path, and "
                               "HBM runs at ~0.4 of peak (see 'hbm'); the binding roof is VALU "
                               "(DESIGN.md 2.1, profiles/r01_ubench_*)"),
                "achieved": valu,
                "peak": VALU_PEAK_TOPS,
                "unit": "T int32 ops/s",
                "frac": valu / VALU_PEAK_TOPS,
                "traffic": traffic,
                "valu_busy": valu_busy,
                "power": power,
                "kernel_ms": kern_ms,
                "kernel_ms_ranks": {"min": min(k1_ms_ranks), "max": max(k1_ms_ranks),
                                    "per_rank": k1_ms_ranks},
                "work_per_file": {"message_bytes": MSG_BYTES, "compressions": COMPRESSIONS,
                                  "spec_ops_per_compression": SPEC_OPS},
                # secondary views of the same kernel time
                "hbm": {"achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS,
                        "algorithmic_bytes_per_launch": F * MSG_BYTES,
                        "traffic_over_algorithmic": (traffic / (F * MSG_BYTES)) if traffic else None},
                "int_ops": {"achieved_spec_tops": valu, "achieved_hw_instr_tops": valu_hw,
                            "peak_full_rate_tops": VALU_PEAK_TOPS},
            },
            "sustained": sustained,
            "e2e": e2e,
            "group": ({
                # the N > 1 grouping: partition + fixed-capacity RCCL all-to-all + grouping of
                # the received keys + mirror all-to-all, one step alone after the timed region
                "mode": "exchange", "ms": exchange_ms, "keys_per_rank": F, "keys": world * F,
                "keys_per_s": world * F / (exchange_ms / 1e3), "phases_ms": exchange_phases,
                "objects": objects, "timed_steps_overflowed": n_overflow,
                "note": "max over ranks; inside the steps it overlaps the next K1 on a side stream"}
                if sharded else None) if group_ms is None else {
                "fused": fused_rec,
                # Object grouping of one step's keys alone (region partition + LDS hash
                # min), HIP events on the stream it runs on, after the timed region: `ms` per
                # call over 10 back-to-back calls, `ms_each_synced` one call at a time
                "ms": group_ms, "ms_each_synced": group_ms_sync, "keys": F,
                "algorithmic_bytes_per_key": group_bytes_per_key(F),
                "achieved_gb_s": F * group_bytes_per_key(F) / (group_ms / 1e3) / 1e9,
                "hbm_frac": F * group_bytes_per_key(F) / (group_ms / 1e3) / 1e9 / HBM_PEAK_GBS,
                "rank_share_config4": {
                    "keys": 12_500_000, "dup_keys": 3_750_000, "objects": group12_objects,
                    "objects_expected": 12_500_000 - 3_750_000,
                    "ms": group12_ms, "algorithmic_bytes_per_key": group_bytes_per_key(12_500_000),
                    "hbm_frac": 12_500_000 * group_bytes_per_key(12_500_000) / (group12_ms / 1e3)
                                / 1e9 / HBM_PEAK_GBS,
                    "lsd_sort": lsd12},
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if worker is not None:
        worker.shutdown()
    if sharded:
        dist.destroy_process_group()


def lsd_sort_leg(eng, keys, rep, objects, stream):
    """The north star's dedup primitive on config 4's rank share: the stable LSD radix sort of
    the 12.5 M keys (K4, 8 x 8-bit passes) and the sort + run heads (K4 + K5), HIP events on
    the stream they run on — "HBM GB/s for the sort": algorithmic bytes (as implemented: 8 x
    (8 B upsweep read + 24 B key/idx read + write) = 256 B/key for the sort, + run heads 8 and
    emit 16 = 280 with the runs) and the PMC bytes per key of the committed pass
    (profiles/r05/pmc_sort_12p5m.json) over this run's times.  The Object count must equal
    the hash grouping's."""
    import numpy as np
    import torch
    n = int(keys.numel())
    ko = torch.empty_like(keys)
    vo = torch.empty(n, dtype=torch.int32, device=keys.device)
    eng.sort_pairs(keys, None, ko, vo)
    objs = eng.group_sorted(ko, vo, rep)
    t_sort, t_runs = [], []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        eng.sort_pairs(keys, None, ko, vo)
        b.record(stream)
        b.synchronize()
        t_sort.append(a.elapsed_time(b))
        a.record(stream)
        eng.sort_pairs(keys, None, ko, vo)
        eng.group_sorted(ko, vo, rep)
        b.record(stream)
        b.synchronize()
        t_runs.append(a.elapsed_time(b))
    ms_sort, ms_runs = float(np.median(t_sort)), float(np.median(t_runs))
    rec = {"keys": n, "ms_sort": ms_sort, "ms_sort_runs": ms_runs, "objects": objs,
           "objects_equal_hash_grouping": objs == objects,
           "algorithmic_bytes_per_key_sort": 256, "algorithmic_bytes_per_key_sort_runs": 280,
           "achieved_gb_s_sort": n * 256 / (ms_sort / 1e3) / 1e9,
           "hbm_frac_sort": n * 256 / (ms_sort / 1e3) / 1e9 / HBM_PEAK_GBS,
           "hbm_frac_sort_runs": n * 280 / (ms_runs / 1e3) / 1e9 / HBM_PEAK_GBS}
    path = os.path.join(ROOT, "profiles", "r05", "pmc_sort_12p5m.json")
    if os.path.exists(path):
        with open(path) as fh:
            pm = json.load(fh)["lsd"]
        rec["pmc_bytes_per_key_sort_runs"] = pm["measured_b_per_key"]
        rec["pmc_gb_s_sort_runs"] = n * pm["measured_b_per_key"] / (ms_runs / 1e3) / 1e9
        rec["pmc_source"] = "profiles/r05/pmc_sort_12p5m.json (measured_in_this_run: false)"
    return rec


class SmiSampler:
    """rocm-smi socket power and shader clock of THIS rank's card, sampled every ~0.25 s by a
    thread (each sample a `rocm-smi -P -g --showbus --json` child process: it reads the SMI,
    no HIP) until stop(); the card is matched by PCI bus number, and with several cards and
    no match nothing is reported (never another card's numbers)."""

    def __init__(self, props, settle_s: float = 1.0):
        import threading
        self.bus = getattr(props, "pci_bus_id", None)
        self.settle = settle_s
        self.samples = []
        self.t0 = time.perf_counter()
        self._stop = threading.Event()
        self._th = threading.Thread(target=self._loop, daemon=True)
        self._th.start()

    def _sample(self):
        import re
        import subprocess
        try:
            r = subprocess.run(["rocm-smi", "-P", "-g", "--showbus", "--json"], capture_output=True,
                               text=True, timeout=10)
            d = json.loads(r.stdout)
        except (OSError, ValueError, subprocess.SubprocessError):
            return None
        if not isinstance(d, dict):
            return None
        cards = [v for k, v in d.items() if str(k).startswith("card") and isinstance(v, dict)]
        pick = None
        for c in cards:
            for k, v in c.items():
                m = re.search(r"[0-9a-fA-F]{4}:([0-9a-fA-F]{2}):", str(v)) if "bus" in k.lower() else None
                if m and self.bus is not None and int(m.group(1), 16) == self.bus:
                    pick = c
        if pick is None and len(cards) == 1:
            pick = cards[0]
        if pick is None:
            return None
        power = sclk = None
        for k, v in pick.items():
            kl = k.lower()
            if "power" in kl and power is None:
                m = re.search(r"[\d.]+", str(v))
                power = float(m.group()) if m else None
            if "sclk" in kl and sclk is None:
                m = re.search(r"(\d+)\s*mhz", str(v).lower())
                sclk = float(m.group(1)) if m else None
        return power, sclk

    def _loop(self):
        while not self._stop.is_set():
            t = time.perf_counter() - self.t0
            smp = self._sample()
            if smp is not None:
                self.samples.append((t, *smp))
            self._stop.wait(0.25)

    def stop(self):
        import statistics
        self._stop.set()
        self._th.join(timeout=15)
        settled = [x for x in self.samples if x[0] >= self.settle]
        pw = [x[1] for x in settled if x[1] is not None]
        ck = [x[2] for x in settled if x[2] is not None]
        if not pw and not ck:
            return None
        return {"power_w_median": statistics.median(pw) if pw else None,
                "sclk_mhz_median": statistics.median(ck) if ck else None,
                "samples": len(settled), "pci_bus": self.bus}


def valu_power_evidence(kname: str, F: int, kern_ms: float, sustained, live):
    """(roofline.valu_busy, roofline.power).  Counter and ceiling figures are read from the
    committed same-session file profiles/r05_valu_power.json (tools/valu_power.py) and marked
    measured_in_this_run = false with that session's id; `live` (rocm-smi during this run's
    sustained steps) is this run's own, and the frac against the compute-only ceiling is
    given both ways: same-session (probe clock) and live (this run's clock)."""
    path = os.path.join(ROOT, "profiles", "r05_valu_power.json")
    if not os.path.exists(path):
        return None, ({"live": live, "measured_in_this_run": True} if live else None)
    with open(path) as fh:
        vp = json.load(fh)
    prov = {"measured_in_this_run": False, "session": vp.get("session"),
            "source": "profiles/r05_valu_power.json (tools/gpu_r5_valu_power.sh: rocprofv3 --pmc, "
                      "tools/ubench_k1 compute-only loop and tools/clock_probe.py in ONE gpurun session)"}
    valu = None
    rec = (vp.get("pmc") or {}).get(kname)
    if rec:
        valu = {"valu_busy": rec["valu_busy"],
                "instr_rate_t_per_s": rec["instr_rate_t_per_s"],
                "instr_rate_frac_of_peak": rec["instr_rate_t_per_s"] / VALU_PEAK_TOPS,
                "instr_per_wave": rec["valu_instr_per_wave"], "clock_ghz": rec.get("clock_ghz"),
                "spec_ops_t_per_s_this_run": F * COMPRESSIONS * SPEC_OPS / (kern_ms / 1e3) / 1e12,
                "note": "instr_rate = SQ_INSTS_VALU x 64 lanes / the PMC pass's mean kernel time "
                        "(every VALU instruction of the kernel, against the 78.6 T lane-op/s "
                        "full-rate peak); valu_busy = rocprof VALUBusy = SQ_ACTIVE_INST_VALU x 4 / "
                        "(1,024 SIMDs x GRBM_GUI_ACTIVE/8).  The ARX mix issues at ~4 cycles per "
                        "wave64 instruction (DESIGN.md 2.1), which is what VALUBusy charges",
                **prov}
    ceil = vp.get("ceiling") or {}
    power = {"session": {k: vp.get(k) for k in ("clock_probe",)}, **prov}
    fpc = ceil.get("files_per_cycle")
    if fpc:
        power["ceiling_files_per_cycle"] = fpc
        power["session_frac_of_capped_ceiling"] = ceil.get("k1_frac_of_capped_ceiling")
    if live:
        power["live"] = dict(live, measured_in_this_run=True)
        if fpc and live.get("sclk_mhz_median") and sustained:
            cap = fpc * live["sclk_mhz_median"] * 1e6
            power["live"]["ceiling_files_per_s_at_live_clock"] = cap
            power["live"]["sustained_frac_of_capped_ceiling"] = (
                sustained["value"] / sustained.get("n_gpus", 1) / cap)
    return valu, power


def fail(msg: str) -> None:
    print(msg, file=sys.stderr, flush=True)
    sys.exit(2)


def visible_gpus(topology: str = "/sys/class/kfd/kfd/topology/nodes") -> int:
    """GPUs this process would see, counted WITHOUT touching HIP: the KFD topology's GPU
    nodes (a non-zero gfx_target_version; CPU nodes have 0), narrowed by
    ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES as the runtime would.
    No KFD topology = no ROCm GPU."""
    import glob
    gpus = 0
    for p in glob.glob(os.path.join(topology, "*", "properties")):
        try:
            with open(p) as fh:
                for line in fh:
                    k, _, v = line.partition(" ")
                    if k == "gfx_target_version" and int(v) != 0:
                        gpus += 1
        except (OSError, ValueError):
            continue
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            gpus = min(gpus, len([x for x in v.split(",") if x.strip()]))
    return gpus


def spawn_ranks(n: int, rehearsal: bool) -> int:
    """Run this bench as n ranks (one process per GPU) under torch.distributed.run, the way
    the driver launches it, and return the launcher's exit status.  The parent never
    initialises the GPU (it counts devices from the KFD topology in sysfs, visible_gpus) and
    does not exec: it starts the launcher as a child, lets rank 0's one JSON line through to
    its own stdout and exits with the child's code."""
    import socket
    import subprocess
    have = visible_gpus()
    if have < n and not rehearsal:
        print(f"bench: --gpus {n} needs {n} visible GPUs, found {have} "
              "(SD_BENCH_ONE_DEVICE=1 rehearses the N > 1 path on one GPU)",
              file=sys.stderr, flush=True)
        return 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.run(cmd).returncode


def e2e_leg(eng, content, sizes, keys, args, world, rank, dev, dist):
    """BASELINE config 3 as worded (PCIe-inclusive): the job's 10.49M sampled files (split
    over the ranks) streamed from pinned host memory through sd_cas_hash_sampled_host_ring —
    H2D of batch k+1 on the side stream overlapping K1 on batch k.  The host ring holds the
    first `ring` files of the resident batch (copied down once, untimed) and is reused
    cyclically: every file's 57,344 B cross PCIe.  Parity: each ring pass equals the
    resident K1 keys of the same files."""
    import numpy as np
    import torch
    F = content.shape[0]
    n = max(1, args.e2e_files // world)
    ring = min(max(16_384, args.e2e_ring // world), F, n)
    pinned = torch.empty((ring, 57344), dtype=torch.uint8, pin_memory=True)
    pinned.copy_(content[:ring])
    hs = sizes[:ring].cpu().numpy().view(np.uint64)
    hsz = np.resize(hs, n)
    want = keys[:ring].cpu().numpy().view(np.uint64)
    eng.hash_sampled_host_ring(pinned.data_ptr(), ring, hsz[:65536])  # warm: staging buffers
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    got = eng.hash_sampled_host_ring(pinned.data_ptr(), ring, hsz)
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    parity = bool((got[:ring] == want).all() and (got == np.resize(want, n)).all())
    ok = torch.tensor([1 if parity else 0], dtype=torch.int64, device=dev)
    if dist is not None:
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    del pinned
    total = n * world
    h2d = total * 57344 / dt / 1e9
    return {"files": total, "files_per_gpu": n, "seconds": dt, "value": total / dt,
            "unit": "cas_ids/s", "hashed_gb_per_s": total * MSG_BYTES / dt / 1e9,
            "h2d_gb_per_s": h2d, "pcie_peak_gb_per_s_per_gpu": PCIE_PEAK_GBS,
            "pcie_frac": h2d / world / PCIE_PEAK_GBS, "ring_files": ring,
            "parity_vs_resident_k1": bool(ok.item()),
            "note": "PCIe-inclusive: pinned host ring -> HBM (side stream) overlapped with K1; "
                    "strong scaling of the 10.49M-file job over the ranks"}


def cpu_threads(world: int) -> int:
    """Host threads for the CPU baseline beside an N-GPU line: the WHOLE node's share, never
    one GPU's.  SD_CPU_BASELINE_THREADS if set; else OMP_NUM_THREADS x world when
    OMP_NUM_THREADS grants more than one (the GPU box sets it to its per-GPU core share, 16),
    else 16 x world; both capped by the cores this process may run on (its affinity mask).
    torch.distributed.run sets OMP_NUM_THREADS=1 for its workers when the caller left it
    unset, which would time the node's CPU on one core beside an N-GPU line."""
    v = int(os.environ.get("SD_CPU_BASELINE_THREADS", "0") or 0)
    if v > 0:
        return v
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = os.cpu_count() or 1
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    per_gpu = omp if omp > 1 else 16
    return max(1, min(avail, per_gpu * max(1, world)))


def cpu_model() -> str | None:
    """The host CPU's model name (/proc/cpuinfo), for the baseline's record."""
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.lower().startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(content, sizes, keys, seconds: float):
    """Oracle AVX-512 path on the host cores over a bounded sample of the same files."""
    import numpy as np

    from oracle.pyoracle import Oracle
    orc = Oracle()
    threads = cpu_threads(int(os.environ.get("WORLD_SIZE", "1")))
    m = min(content.shape[0], 16 * 4096)
    host = content[:m].cpu().numpy()
    hs = sizes[:m].cpu().numpy().view(np.uint64)
    gk = keys[:m].cpu().numpy().view(np.uint64)
    # calibrate, then hash whole passes over the sample for ~`seconds`
    t0 = time.perf_counter()
    k = orc.fast_cas_keys_strided(host.reshape(-1), 57344, 57344, hs, threads)
    one = time.perf_counter() - t0
    parity = bool((k == gk).all())
    reps = max(1, int(seconds / max(one, 1e-3)))
    t0 = time.perf_counter()
    for _ in range(reps):
        orc.fast_cas_keys_strided(host.reshape(-1), 57344, 57344, hs, threads)
    dt = time.perf_counter() - t0
    files = reps * m
    # reference-faithful mode: one hashing thread, as one job's join_all
    m1 = min(m, 2048)
    t0 = time.perf_counter()
    r1 = 0
    while time.perf_counter() - t0 < 1.0:
        orc.fast_cas_keys_strided(host[:m1].reshape(-1), 57344, 57344, hs[:m1], 1)
        r1 += 1
    one_thread = r1 * m1 / (time.perf_counter() - t0)
    official = official_c_leg(host, hs, gk, threads, seconds / 2)
    port_value = files / dt
    best = max(port_value, official["value"]) if official and official.get("parity_vs_gpu") else port_value
    return {"value": best, "unit": "cas_ids/s", "hashed_gb_per_s": best * MSG_BYTES / 1e9,
            "value_port": port_value,
            "value_rule": "the faster of the AVX-512 port and the official C library leg (official_c)",
            "cores": threads, "kind": "port", "value_1thread": one_thread,
            "official_c": official,
            "cpu_model": cpu_model(), "cpus_online": os.cpu_count(),
            "threads_rule": "cpu_threads(world): min(affinity, OMP_NUM_THREADS (or 16) x n_gpus)",
            "threads_override": os.environ.get("SD_CPU_BASELINE_THREADS") or None,
            "simd": "avx512 16-lane" if orc.has_simd() else "scalar",
            "sample": f"{reps} passes over the first {m} files of the bench batch (hashing only, "
                      f"messages pre-gathered in DRAM), {dt:.1f}s",
            "parity_vs_gpu": parity}


def official_c_leg(host, hs, gk, threads: int, seconds: float):
    """The reference's per-file sequence (cas.rs:23-62: Hasher::new, update(le64(size)),
    update(content), finalize) run by the BLAKE3 team's own C implementation, dlopened from
    ROCm's libclang-cpp.so (oracle/ext_b3.c), files statically partitioned over the same
    threads; None if the library is absent."""
    try:
        from oracle.pyoracle import ExtBlake3
        ext = ExtBlake3()
    except Exception:  # no libclang-cpp.so, or the harness could not be built: no leg
        return None
    m = host.shape[0]
    t0 = time.perf_counter()
    k = ext.cas_keys_strided(host.reshape(-1), 57344, 57344, hs, threads)
    one = time.perf_counter() - t0
    reps = max(1, int(seconds / max(one, 1e-3)))
    t0 = time.perf_counter()
    for _ in range(reps):
        ext.cas_keys_strided(host.reshape(-1), 57344, 57344, hs, threads)
    dt = time.perf_counter() - t0
    m1 = min(m, 1024)
    t1 = time.perf_counter()
    r1 = 0
    while time.perf_counter() - t1 < 0.5:
        ext.cas_keys_strided(host[:m1].reshape(-1), 57344, 57344, hs[:m1], 1)
        r1 += 1
    return {"value": reps * m / dt, "unit": "cas_ids/s", "threads": threads,
            "value_1thread": r1 * m1 / (time.perf_counter() - t1),
            "library": f"BLAKE3 C {ext.version()} (llvm_blake3_* in /opt/rocm/lib/llvm/lib/libclang-cpp.so)",
            "sample": f"{reps} passes over the same {m} files, {dt:.1f}s",
            "parity_vs_gpu": bool((k == gk).all())}


if __name__ == "__main__":
    main()
