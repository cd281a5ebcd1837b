"""Headline benchmark: Mrays/s (closest + shadow) of the path-tracing hot path
on the procedural 1M-triangle scene, 1920x1080, 256 spp (BASELINE.json
configs[2]; configs[3] when launched on N GPUs).

One step = one whole frame: every rank renders the tiles t with
t % world == rank (yk_render_shard), the film sums are reduced to rank 0 over
RCCL (torch.distributed "nccl") and rank 0 normalises the frame
(yk_film_resolve). Total work is fixed as N grows ("scaling": "strong").

  python bench.py [--gpus N] [--steps K] [--warmup W]

Under torch.distributed.run every process is one rank. Started directly with
--gpus N > 1, bench.py starts the N rank processes itself (launch_ranks)
before it touches a GPU, and exits non-zero if any of them fails.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from core_amd import _abi as A  # noqa: E402
from core_amd.device import Device  # noqa: E402
from core_amd.scene import probe_scene  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
L2_PEAK_GBS = 34500.0  # aggregate L2 bandwidth, 8 XCDs (MI355X_MICROARCH.md, "L2 (per XCD)")
LDS_PEAK_GBS = 150000.0  # aggregate LDS read bandwidth, ds_read_b64/b128 on every CU (MI355X_MICROARCH.md §LDS)


def algorithmic_bytes(rays, nodes, tris, out_bytes):
    """Bytes one traversal launch must move if nothing were cached: the ray
    (32 B) and its result, one 8-B node per visit, and per triangle test the
    9 vertex floats (36 B) plus its 4-B leaf-list entry."""
    return rays * (32 + out_bytes) + 8 * nodes + 40 * tris


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="bumpy", choices=["bumpy", "hair", "cornell"],
                    help="bumpy: the 1M-tri headline probe (configs[2]); hair: the C5 10M-tri strand scene; "
                         "cornell: configs[1] (36 tris, pass --width 1024 --height 1024 --spp 64)")
    ap.add_argument("--strands", type=int, default=200000, help="hair: strands (x50 tris each at 9 points)")
    ap.add_argument("--strand-points", type=int, default=9)
    ap.add_argument("--nu", type=int, default=1000, help="sphere segments (1000x501 -> 1,000,002 tris)")
    ap.add_argument("--nv", type=int, default=501)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--integrator", default="path", choices=["path", "photon"],
                    help="path: the headline pathtracing integrator; photon: photonmapping with final gathering "
                         "(the photon maps are built once before timing, like the kd-tree)")
    ap.add_argument("--photons", type=int, default=100000, help="photon: diffuse photons (reference default)")
    ap.add_argument("--fg-samples", type=int, default=32, help="photon: final-gather paths per hit (default 32)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target length of the CPU baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--gpu-tree", action="store_true",
                    help="replace the reference kd-tree by the device-built binned-SAH tree (yk_device_build_tree, "
                         "documented tie-break; not the parity default)")
    ap.add_argument("--traffic", default=None,
                    help="PMC HBM-traffic summary (tools/pmc_traffic.py output of the one-pipe frame) to attach; "
                         "default profiles/traffic.json (bumpy), traffic_hair.json (hair), traffic_c2.json "
                         "(cornell), path tracing only")
    ap.add_argument("--pipes", type=int, default=0,
                    help="batch pipelines of the timed frames (default: libyk's 4; 1 serialises the kernels)")
    ap.add_argument("--no-roofline-frame", action="store_true",
                    help="skip the extra serialised frame the roofline line is measured on")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="film-reduce backend for N > 1: nccl (RCCL over xGMI, one GPU per rank) or gloo (host "
                         "copies; lets N ranks share one GPU, for tests)")
    args = ap.parse_args()
    if args.pipes:
        os.environ["YK_PIPES"] = str(args.pipes)

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: start the N rank processes here, before this process
        # touches the GPU (torch is imported, no device call made yet)
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    fail = os.environ.get("YK_BENCH_FAIL_RANK")  # test hook: this rank exits at once (launcher failure path)
    if fail is not None and int(fail) == rank:
        raise SystemExit(3)
    dist = None
    gloo = args.backend == "gloo"
    if world > 1:
        import torch.distributed as dist
        if gloo:
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        # ranks beyond the visible GPUs share them (gloo test runs on one GPU)
        local = local % max(1, torch.cuda.device_count())

    t_build = time.perf_counter()
    if rank == 0:
        print(f"[bench] building {args.scene} scene + kd-tree on the host", file=sys.stderr, flush=True)
    if args.scene == "hair":
        scene, p = probe_scene("hair", args.width, args.height, args.strands, args.strand_points)
    elif args.scene == "cornell":  # BASELINE configs[1]: path_samples 1, bounces 4, raydepth 2
        scene, p = probe_scene("cornell_pt", args.width, args.height)
    else:
        scene, p = probe_scene("bumpy", args.width, args.height, args.nu, args.nv)
    t_build = time.perf_counter() - t_build
    info = scene.info()
    p.aa_samples = args.spp
    dev = Device(local)
    dev.upload(scene)
    tree_info = dev.build_tree(scene) if args.gpu_tree else None
    small = small_scene_bytes(dev)
    pm_info = None
    if args.integrator == "photon":  # photonIntegrator_t::preprocess, once per scene (not timed)
        p.integrator = A.YK_INTEGRATOR_PHOTON
        p.photon.photons = args.photons
        p.photon.fg_samples = args.fg_samples
        pm_info = dev.photon_build(p)
    film = dev.new_film(p)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    red_ev = []  # (start, end) CUDA events around every film reduce of the timed steps

    def step(st, ev=None):
        film.zero_()
        dev.render_shard(p, film, rank, world, st)
        if dist is not None:
            if ev is not None:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
            if gloo:  # gloo reduces host tensors: device -> host, reduce, host -> device
                h = film.cpu()
                dist.reduce(h, dst=0)
                if rank == 0:
                    film.copy_(h)
            else:
                dist.reduce(film, dst=0)
            if ev is not None:
                e1.record()
                ev.append((e0, e1))
        if rank == 0:
            rgba = dev.film_resolve(p, film)
            return rgba
        return None

    for _ in range(args.warmup):
        step(A.yk_stats())
    st = A.yk_stats()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(st, red_ev)
    barrier()
    elapsed = time.perf_counter() - t0
    # RCCL film reduce per step (inside the timed region; 0 on one GPU)
    ms_reduce = sum(a.elapsed_time(b) for a, b in red_ev) / max(args.steps, 1)

    # whole-job numbers: sum the work, take the slowest rank's time
    work = torch.tensor([st.closest_rays, st.shadow_rays, st.closest_nodes, st.closest_tris, st.shadow_nodes,
                         st.shadow_tris, st.closest_launches, st.shadow_launches, st.camera_samples],
                        dtype=torch.float64, device="cuda")
    kern = torch.tensor([st.ms_closest, st.ms_shadow], dtype=torch.float64, device="cuda")
    tmax = torch.tensor([elapsed, ms_reduce], dtype=torch.float64, device="cuda")
    if dist is not None:
        if gloo:
            work, kern, tmax = work.cpu(), kern.cpu(), tmax.cpu()
        dist.all_reduce(work)
        dist.all_reduce(kern)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    w = work.cpu().numpy()
    ms_c, ms_s = kern.cpu().numpy()
    elapsed, ms_reduce = (float(x) for x in tmax.cpu().numpy())
    rays = w[0] + w[1]
    value = rays / elapsed / 1e6

    # Roofline frame: one more frame (not part of `value`) with the kernels
    # serialised on one pipeline (YK_PIPES=1), so that each traversal
    # launch's HIP-event duration is its own and not time shared with the
    # other pipes' kernels. rocprofv3 --kernel-trace --stats of
    # `bench.py --pipes 1` gives the same per-launch averages (profiles/).
    rst = None
    if not args.no_roofline_frame:
        prev = os.environ.get("YK_PIPES")
        os.environ["YK_PIPES"] = "1"
        rst = A.yk_stats()
        barrier()
        step(rst)
        barrier()
        if prev is None:
            del os.environ["YK_PIPES"]
        else:
            os.environ["YK_PIPES"] = prev

    if rank != 0:
        dist.destroy_process_group()
        return

    roofline = roofline_line(args, w, ms_c, ms_s, rst, elapsed, pm_info is None, small, shadow_split(dev, p))

    cpu = None
    if not args.no_cpu:
        cpu = cpu_baseline(scene, p, args.cpu_seconds)

    out = {
        "metric": {"bumpy": "Mrays/s (primary+shadow), 1M-tri scene",
                   "hair": "Mrays/s (primary+shadow), 10M-tri hair scene (C5 shape)",
                   "cornell": "Mrays/s (primary+shadow), Cornell box (configs[1])"}[args.scene] +
                  (", photon mapping" if pm_info is not None else ""),
        "value": round(value, 3),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "ms_reduce": round(ms_reduce, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": {"bumpy": "synthetic: procedural displaced sphere + floor",
                 "hair": f"synthetic: {args.strands} curve strands x {args.strand_points} points on a sphere + floor",
                 "cornell": "the reference-fixture Cornell box (tests/golden/gen)"}[args.scene] +
                f", {info.ntris} tris, " + (f"kd-tree built on the device ({tree_info.ms_build:.1f} ms, not timed; "
                                           f"the reference tree {t_build:.1f} s on host first)" if tree_info is not None
                                           else f"kd-tree built on host ({t_build:.1f} s, not timed)"),
        "config": {"workload": f"{args.scene} {info.ntris} tris, " +
                               (f"pathtracing bounces {p.bounces}, " if pm_info is None else
                                f"photonmapping {p.photon.photons} photons, final gather {p.photon.fg_samples} paths "
                                f"x {p.photon.fg_bounces} bounces, search {p.photon.search}, ") +
                               f"{p.width}x{p.height}, {p.aa_samples} spp, {info.nlights} area light(s)",
                   "tris": int(info.ntris), "width": p.width, "height": p.height, "spp": p.aa_samples,
                   "parallelism": f"tiles%{world}" if world > 1 else "single",
                   "closest_rays": int(w[0]), "shadow_rays": int(w[1]),
                   "camera_samples": int(w[8]),
                   "per_ray": {"closest_nodes": round(w[2] / max(w[0], 1), 2),
                               "closest_tri_tests": round(w[3] / max(w[0], 1), 2),
                               "shadow_nodes": round(w[4] / max(w[1], 1), 2),
                               "shadow_tri_tests": round(w[5] / max(w[1], 1), 2)}},
        "roofline": roofline,
        "cpu_baseline": cpu,
    }
    if pm_info is not None:
        out["config"]["photon_maps"] = {
            "diffuse_photons": pm_info.diffuse_photons, "radiance_photons": pm_info.radiance_photons,
            "photon_rays": int(pm_info.photon_rays), "preprocess_ms": round(pm_info.ms_total, 1),
            "shoot_ms": round(pm_info.ms_shoot, 1), "pregather_ms": round(pm_info.ms_pregather, 1)}
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def _hook(fn, *args):
    """A read-only query of the test-hooks header, enabled for this call."""
    old = os.environ.get("YK_DEBUG_HOOKS")
    os.environ["YK_DEBUG_HOOKS"] = "1"
    try:
        A.check(fn(*args))
    finally:
        if old is None:
            del os.environ["YK_DEBUG_HOOKS"]
        else:
            os.environ["YK_DEBUG_HOOKS"] = old


def small_scene_bytes(dev):
    """Bytes of the LDS copy of the traversal data when the resident scene runs
    the small-scene kernels (k_trace_*_small), else 0."""
    b = C.c_int64(0)
    _hook(A.lib().yk_debug_small_scene, dev._p, C.byref(b))
    return int(b.value)


def shadow_split(dev, p):
    """True when a render with params p stores split shadow slots (16-B
    direction records, any-hit kernels k_trace_shadow[_small]_split)."""
    v = C.c_int32(0)
    _hook(A.lib().yk_debug_shadow_form, dev._p, C.byref(p), C.byref(v))
    return bool(v.value)


def roofline_line(args, w, ms_c, ms_s, rst, elapsed, pt, small=0, split=False):
    """Roofline of the dominant traversal kernel. Durations come from the
    serialised roofline frame (rst) when it ran, else from the timed frames'
    HIP events (overlapped by the other pipes: a lower bound on the rate).
    small > 0: the scene's traversal data sits in LDS (small-scene kernels),
    so its node / record bytes are LDS reads; the line then also prices them
    against the LDS peak."""
    if rst is not None:
        cnt = [rst.closest_rays, rst.shadow_rays, rst.closest_nodes, rst.closest_tris, rst.shadow_nodes,
               rst.shadow_tris, rst.closest_launches, rst.shadow_launches]
        ms = (rst.ms_closest, rst.ms_shadow)
        timing = "serialised frame (YK_PIPES=1): HIP events around every launch on its stream"
    else:
        cnt = list(w[:8])
        ms = (ms_c, ms_s)
        timing = "timed frames: HIP events around every launch, overlapped by the other pipes"
    sfx = "_small" if small else ""
    kc = dict(name="k_trace_closest" + sfx, launches=cnt[6], ms=ms[0], bytes=algorithmic_bytes(cnt[0], cnt[2], cnt[3], 16))
    # H = 4 B for the shadow result, as SURVEY.md §8(d) prices it (the kernel
    # stores 1 B)
    ks = dict(name="k_trace_shadow" + sfx + ("_split" if split else ""), launches=cnt[7], ms=ms[1], bytes=algorithmic_bytes(cnt[1], cnt[4], cnt[5], 4))
    for k in (kc, ks):
        k["gbs"] = k["bytes"] / (k["ms"] * 1e-3) / 1e9 if k["ms"] > 0 else 0.0
        k["avg_ms"] = k["ms"] / max(k["launches"], 1)
    dom, other = (kc, ks) if kc["ms"] >= ks["ms"] else (ks, kc)
    traffic = traffic_raw = traffic_note = None
    tfile = args.traffic or (os.path.join(ROOT, "profiles", {"bumpy": "traffic.json", "hair": "traffic_hair.json",
                                                             "cornell": "traffic_c2.json"}[args.scene]) if pt else "")
    key = "closest" if dom is kc else "shadow"
    if tfile and os.path.isfile(tfile):  # PMC summary of this scene's one-pipe PT frame
        with open(tfile) as f:
            tj = json.load(f)
        # only a pass over the same launch partition as the roofline frame
        # (one pipe: same batches, same launches) is comparable per launch
        if key in tj and (rst is None or int(tj[key].get("launches", -1)) == int(dom["launches"])):
            traffic = tj[key].get("hbm_bytes_per_launch")
            traffic_raw = tj[key].get("hbm_bytes_per_launch_raw")
            traffic_note = tj.get("source")
    # the HBM roofline, unless the algorithmic rate is above the HBM peak: then
    # the re-reads are served by L2 / the Infinity Cache and L2 bandwidth (34.5
    # TB/s aggregate, MI355X_MICROARCH.md "L2 (per XCD)") is the bound
    l2_bound = dom["gbs"] > HBM_PEAK_GBS
    peak = L2_PEAK_GBS if l2_bound else HBM_PEAK_GBS
    out = {"bound": "l2" if l2_bound else "hbm", "achieved": round(dom["gbs"], 2), "peak": peak, "unit": "GB/s",
           "frac": round(dom["gbs"] / peak, 4), "traffic": traffic,
           "kernel": dom["name"], "avg_launch_ms": round(dom["avg_ms"], 4), "launches": int(dom["launches"]),
           "algorithmic_bytes_per_launch": round(dom["bytes"] / max(dom["launches"], 1)), "timing": timing,
           "other_kernel": {"name": other["name"], "achieved": round(other["gbs"], 2),
                            "avg_launch_ms": round(other["avg_ms"], 4),
                            "frac": round(other["gbs"] / HBM_PEAK_GBS, 4)}}
    if traffic:
        # counter view: measured HBM bytes per launch of the same launch
        # partition over the same launch duration; (2*FETCH + WRITE) with the
        # guide's gfx950 FETCH correction, and the raw (FETCH + WRITE) beside
        # it -- the correction is calibrated on wide streaming reads only
        out["traffic_raw"] = traffic_raw
        out["traffic_gbs"] = round(traffic / (dom["avg_ms"] * 1e-3) / 1e9, 2)
        out["traffic_gbs_raw"] = round((traffic_raw or 0) / (dom["avg_ms"] * 1e-3) / 1e9, 2)
        out["frac_traffic"] = round(out["traffic_gbs"] / HBM_PEAK_GBS, 4)
        out["traffic_source"] = traffic_note
    out["hbm"] = {"peak": HBM_PEAK_GBS, "frac": round(dom["gbs"] / HBM_PEAK_GBS, 4)}
    out["l2"] = {"peak": L2_PEAK_GBS, "frac": round(dom["gbs"] / L2_PEAK_GBS, 4)}
    if small:
        note = "algorithmic bytes: the node / record bytes among them are LDS reads here, not HBM or L2 traffic"
        out["hbm"]["note"] = note
        out["l2"]["note"] = note
        out["lds"] = {"peak": LDS_PEAK_GBS, "frac": round(dom["gbs"] / LDS_PEAK_GBS, 4), "scene_copy_bytes": small,
                      "note": "traversal data (node packets, triangle records) copied to LDS once per 4-wave "
                              "workgroup: the per-node / per-test bytes are LDS reads, only rays and results "
                              "cross HBM"}
    # all traversal bytes of the timed frames over their wall time
    out["traversal_achieved_wall"] = round((algorithmic_bytes(w[0], w[2], w[3], 16) +
                                            algorithmic_bytes(w[1], w[4], w[5], 4)) / elapsed / 1e9, 2)
    return out


def launch_ranks(n):
    """Start N rank processes of this same command line (RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_ADDR / MASTER_PORT set, as torch.distributed.run sets
    them) and wait for them. Rank 0 prints the JSON line to the inherited
    stdout. Returns 0 when every rank exits 0; when one fails, the others are
    terminated and its exit code is returned. The multi-GPU split this drives
    replaces the reference's render thread pool (integrator.cc:177-211)."""
    import signal
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))

    def stop(*_):
        for q in procs:
            if q.poll() is None:
                q.terminate()
        for q in procs:
            try:
                q.wait(timeout=20)
            except subprocess.TimeoutExpired:
                q.kill()
                q.wait()

    signal.signal(signal.SIGTERM, lambda *a: (stop(), sys.exit(143)))
    rc = 0
    live = list(procs)
    while live:
        for q in list(live):
            code = q.poll()
            if code is None:
                continue
            live.remove(q)
            if code != 0:
                print(f"[bench] rank {procs.index(q)} exited with {code}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                stop()
                return code if code > 0 else 128 - code
        time.sleep(0.2)
    return rc


def host_threads():
    """Host cores this process may use: its CPU affinity, capped by
    OMP_NUM_THREADS where the box sets it to the job's CPU share."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = os.environ.get("OMP_NUM_THREADS")
    if cap and cap.isdigit() and int(cap) > 0:
        n = min(n, int(cap))
    return max(1, n)


def cpu_baseline(scene, p, seconds):
    """The oracle (the C restatement of the reference's CPU path) on all host
    cores, on a bounded centred crop of the same frame: like the reference's
    tiledIntegrator_t::render (integrator.cc:177-211), every thread renders
    tiles, here the shards t % (4 threads) == k. The crop is sized from a
    1-thread probe to about `seconds` of wall time."""
    from concurrent.futures import ThreadPoolExecutor
    sys.path.insert(0, ROOT)
    from oracle.oracle import Oracle
    orc = Oracle(scene)
    q = A.yk_render_params.from_buffer_copy(p)
    if q.integrator == A.YK_INTEGRATOR_PHOTON:
        orc.photon_build(q)  # the oracle's own preprocess (not timed, like the device's)
    q.width, q.height = 16, 16
    q.xstart, q.ystart = p.width // 2, p.height // 2
    t0 = time.perf_counter()
    orc.render(q)  # also initialises the oracle's shared tables before the threads start
    probe = time.perf_counter() - t0
    nt = host_threads()
    # grow the crop to ~`seconds` of wall time on nt threads (square, centred)
    px = max(256, int(16 * 16 * seconds * nt / max(probe, 1e-3)))
    side = int(np.sqrt(px))
    q.width, q.height = min(side, p.width), min(side, p.height)
    q.xstart, q.ystart = (p.width - q.width) // 2, (p.height - q.height) // 2
    nsh = 4 * nt
    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=nt) as ex:  # ctypes releases the GIL inside orc_render_shard
        res = list(ex.map(lambda k: orc.render_shard(q, k, nsh)[1], range(nsh)))
    dt = time.perf_counter() - t0
    r = sum(c["closest"] + c["shadow"] for c in res)
    return {"value": round(r / dt / 1e6, 4), "unit": "Mrays/s", "cores": nt, "kind": "port",
            "sample": f"oracle on {nt} threads ({nsh} tile shards): {q.width}x{q.height} crop at "
                      f"({q.xstart},{q.ystart}) of the same frame, {p.aa_samples} spp, {r} rays in {dt:.1f} s"}


if __name__ == "__main__":
    main()
