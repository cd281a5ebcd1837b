"""Packet-traversal simulator (tools only): replays the headline frame's ray
populations of a few pixels through the reference kd-tree (kdtree.cc:675-947
restated per lane, float32) and through a wave-packet schedule in which the
64 lanes of a wave walk ONE node stream -- every lane keeps its own entry /
exit / stack state and makes the reference's decisions, the packet visits the
union of the lanes' nodes in an order consistent with every lane's own order
(left-first or right-first by majority, a third visit for the minority that
crosses the other way). Reports per packet: node visits of the packet against
the lanes' summed visits, leaf visits, and checks that every lane saw exactly
its own node sequence.
  python tools/packet_sim.py [--pixels N] [--kind shadow0|camera|shadow1]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

f32 = np.float32


class Tree:
    def __init__(self, ex):
        self.n = ex["nodes"]
        self.leaf = ex["leaf_prims"]
        self.tv = ex["tri_verts"]
        self.bound = ex["bound"]

    def interior(self, i):
        return (int(self.n[i, 1]) & 3) != 3

    def axis(self, i):
        return int(self.n[i, 1]) & 3

    def split(self, i):
        return self.n[i, 0:1].view(np.float32)[0]

    def right(self, i):
        return int(self.n[i, 1]) >> 2

    def refs(self, i):
        cnt = int(self.n[i, 1]) >> 2
        w0 = int(self.n[i, 0])
        if cnt == 0:
            return []
        if cnt == 1:
            return [w0]
        return [int(p) for p in self.leaf[w0:w0 + cnt]]


def mt(v, o, d):
    a, b, c = v[0:3], v[3:6], v[6:9]
    e1, e2 = b - a, c - a
    p = np.cross(d, e2).astype(f32)
    det = f32(e1 @ p)
    if det == 0:
        return None
    inv = f32(1) / det
    tv = (o - a).astype(f32)
    u = f32(tv @ p) * inv
    if u < 0 or u > 1:
        return None
    q = np.cross(tv, e1).astype(f32)
    v2 = f32(d @ q) * inv
    if v2 < 0 or u + v2 > 1:
        return None
    return f32(e2 @ q) * inv


class Lane:
    """One ray's reference traversal state (kdtree.cc IntersectS / Intersect)."""

    def __init__(self, T, ray, closest):
        self.T = T
        self.closest = closest
        d = ray[3:6].astype(f32)
        if closest:
            o = ray[0:3].astype(f32)
            self.tmin = f32(ray[6])
            self.dist = f32(np.inf) if ray[7] < 0 else f32(ray[7])
        else:
            o = (ray[0:3] + ray[6] * d).astype(f32)
            self.tmin = f32(0)
            self.dist = f32(np.inf) if ray[7] < 0 else f32(ray[7] - 2 * ray[6])
        self.o, self.d = o, d
        with np.errstate(divide="ignore"):
            self.inv = (f32(1) / d).astype(f32)
        self.Z = self.dist
        self.done = False
        self.hit = False
        self.seq = []
        bb = T.bound
        lo, hi = -f32(1e38), f32(1e38)
        ok = True
        first = True
        for ax in range(3):
            if d[ax] != 0:
                invr = f32(1) / d[ax]
                t0, t1 = (bb[ax] - o[ax]) * invr, (bb[3 + ax] - o[ax]) * invr
                tmn, tmx = (t0, t1) if invr > 0 else (t1, t0)
                if first:
                    lo, hi, first = tmn, tmx, False
                else:
                    lo = lo if tmn < lo else tmn
                    hi = hi if hi < tmx else tmx
                if hi < 0 or lo > self.dist:
                    ok = False
                    break
        if not ok or not (lo <= hi and hi >= 0 and lo <= self.dist):
            self.done = True
            self.want = None
            return
        self.en_t = lo
        self.en_pb = (o + lo * d).astype(f32) if lo >= 0 else o.copy()
        self.ex_t, self.ex_pb, self.ex_far = hi, (o + hi * d).astype(f32), -1
        self.stack = []
        self.want = 0

    def decide(self, node):
        """descent step at interior node: returns (near, pushed far or None)"""
        T = self.T
        ax, s, r = T.axis(node), T.split(node), T.right(node)
        self.seq.append(node)
        enp, exq = self.en_pb[ax], self.ex_pb[ax]
        left_first = enp <= s
        push = (not (exq <= s)) if left_first else (not (s < exq))
        near, far = (node + 1, r) if left_first else (r, node + 1)
        if push:
            t = (s - self.o[ax]) * self.inv[ax]
            self.stack.append((self.ex_t, self.ex_pb, self.ex_far))
            pb = (self.o + t * self.d).astype(f32)
            pb[ax] = s
            self.ex_t, self.ex_pb, self.ex_far = t, pb, far
        self.want = near
        return near, (far if push else None)

    def leaf(self, node):
        T = self.T
        self.seq.append(node)
        for p in T.refs(node):
            t = mt(T.tv[p], self.o, self.d)
            if t is None:
                continue
            if self.closest:
                if t < self.Z and t >= self.tmin:
                    self.Z, self.hit = t, True
            elif t < self.dist and t >= 0:
                self.hit, self.done, self.want = True, True, None
                return
        if self.closest and self.hit and self.Z <= self.ex_t:
            self.done, self.want = True, None
            return
        # pop
        self.en_t, self.en_pb = self.ex_t, self.ex_pb
        if self.ex_far < 0:
            self.done, self.want = True, None
            return
        self.want = self.ex_far
        self.ex_t, self.ex_pb, self.ex_far = self.stack.pop()
        if self.dist < self.en_t:
            self.done, self.want = True, None

    def run(self):
        """per-lane reference traversal"""
        while self.want is not None:
            node = self.want
            if self.dist < self.en_t:
                self.done, self.want = True, None
                break
            while self.T.interior(node):
                node, _ = self.decide(node)
            self.leaf(node)
        return self.seq


def packet(T, rays, closest):
    lanes = [Lane(T, r, closest) for r in rays]
    st = [(0, frozenset(i for i, l in enumerate(lanes) if l.want == 0))]
    visits = leaves = 0
    while st:
        node, mask = st.pop()
        while True:
            act = [i for i in mask if lanes[i].want == node]
            if not act:
                break
            visits += 1
            if not T.interior(node):
                leaves += 1
                for i in act:
                    lanes[i].leaf(node)
                break
            left, right = node + 1, T.right(node)
            lgo, rgo, lr, rl = set(), set(), set(), set()
            for i in act:
                near, far = lanes[i].decide(node)
                (lgo if near == left else rgo).add(i)
                if far == right:
                    lr.add(i)
                elif far == left:
                    rl.add(i)
            if len(lr) >= len(rl):  # left first; right-to-left lanes take a third visit
                if rl:
                    st.append((left, frozenset(rl)))
                if rgo or lr:
                    st.append((right, frozenset(rgo | lr)))
                node, mask = left, frozenset(lgo)
            else:
                if lr:
                    st.append((right, frozenset(lr)))
                if lgo or rl:
                    st.append((left, frozenset(lgo | rl)))
                node, mask = right, frozenset(rgo)
    return lanes, visits, leaves


def block_shadow_rays(orc, p, x0, y0, bw, spp, rng):
    """primary shadow rays of a bw x bw pixel block (camera rays jittered in
    the pixels, hits by the oracle, light points uniform on the 1x1 light)"""
    rays = orc.camera_rays(x0, y0, bw, bw, spp)
    prim, t, _, _, _ = orc.intersect(rays)
    m = prim >= 0
    P = rays[m, 0:3] + t[m, None] * rays[m, 3:6]
    L = np.stack([rng.uniform(-0.5, 0.5, m.sum()), np.full(m.sum(), 3.0), rng.uniform(-0.5, 0.5, m.sum())], 1)
    d = (L - P).astype(np.float32)
    dist = np.linalg.norm(d, axis=1)
    out = np.zeros((m.sum(), 8), np.float32)
    out[:, 0:3], out[:, 3:6], out[:, 6], out[:, 7] = P, d / dist[:, None], 5e-4, dist
    return out, L


def main_block(args):
    """primary shadow rays of one pixel block, in the renderer's order (pixel
    by pixel, samples consecutive) and binned by light cell"""
    from core_amd.scene import probe_scene
    from oracle.oracle import Oracle
    s, p = probe_scene("bumpy", 1920, 1080, 1000, 501)
    T = Tree(s.export())
    orc = Oracle(s)
    rng = np.random.default_rng(args.seed)
    for _ in range(args.pixels):
        x0, y0 = int(rng.integers(300, 1600)), int(rng.integers(250, 900))
        rays, L = block_shadow_rays(orc, p, x0, y0, args.block, args.spp, rng)
        cells = args.cells
        cx = np.clip(((L[:, 0] + 0.5) * cells).astype(int), 0, cells - 1)
        cz = np.clip(((L[:, 2] + 0.5) * cells).astype(int), 0, cells - 1)
        order = np.lexsort((np.arange(len(rays)), cz * cells + cx))
        for name, rr in (("pixel order", rays), ("light-cell order", rays[order])):
            v = lv = u = n = 0
            for g in range(0, min(len(rr), args.max_rays) - 63, 64):
                grp = rr[g:g + 64]
                ref = [Lane(T, r, False).run() for r in grp]
                lv += sum(len(a) for a in ref)
                u += len(set(x for a in ref for x in a))
                n += 1
            print(f"block ({x0},{y0}) {args.block}x{args.block} {len(rays)} rays, {name}: per ray {lv / (64 * n):.1f} "
                  f"node visits, union per 64-ray group {u / n:.1f} ({u / lv * 64:.1f}x a ray)", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--block", type=int, default=0, help="> 0: synthetic primary shadow rays of a pixel block")
    ap.add_argument("--cells", type=int, default=16)
    ap.add_argument("--max-rays", type=int, default=4096)
    ap.add_argument("--pixels", type=int, default=6)
    ap.add_argument("--kind", default="shadow0", choices=["shadow0", "camera", "shadow1", "bounce1"])
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--leaf-stats", action="store_true")
    args = ap.parse_args()
    if args.leaf_stats:
        return leaf_stats(args)
    if args.block:
        return main_block(args)
    from core_amd.scene import probe_scene
    from oracle.oracle import Oracle
    s, p = probe_scene("bumpy", 1920, 1080, 1000, 501)
    T = Tree(s.export())
    orc = Oracle(s)
    rng = np.random.default_rng(args.seed)
    tot = dict(visits=0, lane_visits=0, union=0, leaves=0, lane_leaves=0, rays=0)
    for _ in range(args.pixels):
        x, y = int(rng.integers(300, 1620)), int(rng.integers(250, 1000))
        q = p.copy() if hasattr(p, "copy") else p
        q.aa_samples = args.spp
        q.width, q.height, q.xstart, q.ystart = 1, 1, x, y
        _, log = orc.render_logged(q, x, y)
        kinds = log[:, 0].astype(int)
        cam = np.float32([0, 1.5, -4])
        is_cam = (kinds == 0) & np.all(np.abs(log[:, 2:5] - cam) < 1e-6, axis=1)
        sel = []
        depth = -1
        for k in range(len(log)):
            if is_cam[k]:
                depth = 0
                if args.kind == "camera":
                    sel.append(k)
                continue
            if kinds[k] == 1:
                if (args.kind == "shadow0" and depth == 0) or (args.kind == "shadow1" and depth == 1):
                    sel.append(k)
            elif kinds[k] == 0:
                depth += 1
                if args.kind == "bounce1" and depth == 1:
                    sel.append(k)
        rays = log[sel][:, 2:10]
        closest = args.kind in ("camera", "bounce1")
        for g in range(0, len(rays) - 63, 64):
            grp = rays[g:g + 64]
            ref = [Lane(T, r, closest).run() for r in grp]
            lanes, v, lv = packet(T, grp, closest)
            for a, l in zip(ref, lanes):
                assert a == l.seq, "packet order differs from the lane's own order"
            tot["visits"] += v
            tot["leaves"] += lv
            tot["lane_visits"] += sum(len(a) for a in ref)
            tot["union"] += len(set(n for a in ref for n in a))
            tot["rays"] += len(grp)
            tot["lane_leaves"] += sum(sum(1 for n in a if not T.interior(n)) for a in ref)
        print(f"pixel ({x},{y}): {len(rays)} {args.kind} rays, running: packet visits {tot['visits']} "
              f"vs lane visits {tot['lane_visits']} (union {tot['union']}), packets {tot['rays'] // 64}",
              flush=True)
    npk = max(tot["rays"] // 64, 1)
    print(f"per packet: {tot['visits'] / npk:.1f} packet node visits ({tot['leaves'] / npk:.1f} leaves); "
          f"per ray {tot['lane_visits'] / max(tot['rays'], 1):.1f} node visits "
          f"({tot['lane_leaves'] / max(tot['rays'], 1):.1f} leaves); union per packet {tot['union'] / npk:.1f}")



def leaf_stats(args):
    """empty / non-empty leaves per ray and descent lengths (per-lane reference order)"""
    from core_amd.scene import probe_scene
    from oracle.oracle import Oracle
    s, p = probe_scene("bumpy", 1920, 1080, 1000, 501)
    T = Tree(s.export())
    orc = Oracle(s)
    rng = np.random.default_rng(args.seed)
    x0, y0 = int(rng.integers(300, 1600)), int(rng.integers(250, 900))
    rays, _ = block_shadow_rays(orc, p, x0, y0, 16, 4, rng)
    rays = rays[:2000]
    emp = full = nodes = 0
    runs = []  # consecutive empty leaves between non-empty ones
    for r in rays:
        seq = Lane(T, r, False).run()
        run = 0
        for n in seq:
            nodes += 1
            if T.interior(n):
                continue
            if (int(T.n[n, 1]) >> 2) == 0:
                emp += 1
                run += 1
            else:
                full += 1
                runs.append(run)
                run = 0
    print(f"{len(rays)} shadow rays: per ray {nodes / len(rays):.1f} nodes, {emp / len(rays):.1f} empty leaves, "
          f"{full / len(rays):.1f} non-empty leaves; mean empty run before a non-empty leaf {np.mean(runs):.2f}")


if __name__ == "__main__":
    main()
