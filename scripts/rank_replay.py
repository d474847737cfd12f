"""Per-rank GPU time of the multi-rank unordered pipeline, one rank at a time.

    python scripts/rank_replay.py N P [--k 100]

P loopback ranks (threads) run the unordered pipeline on one GPU once (untimed): every
rank's owned points (after the spatial redistribution), published trees and received
halo points are recorded. Then each rank's own device work is replayed ALONE on the GPU
and timed with events, as it would run on its own MI355X:

  build    index build of the owned points (Hilbert sort, gather, tree, cell grid)
  classify a-priori radius bounds + boundary classification against the other ranks'
           published trees
  local    the local k-NN pass (boundary groups, then interior groups)
  halo     halo filter of the rank's points against the other ranks' published radii
           (what it sends) + the index (tree + grid) of what it received
  requery  flagging + re-query of the groups a received point can reach
  return   the result scatter back to input order (the all-to-all-v itself is xGMI time)

and the halo sizes. Prints one line per rank and a JSON summary (max over ranks). The
collectives' xGMI time is not included (no peers here); see BASELINE.md for the model.
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, ".")
from mpi_cuda_largescaleknn_amd.models import knn_engine as E  # noqa: E402
from mpi_cuda_largescaleknn_amd.ops import kernels as K  # noqa: E402
from mpi_cuda_largescaleknn_amd.parallel import pipelines as PL  # noqa: E402
from mpi_cuda_largescaleknn_amd.parallel.comm import run_loopback  # noqa: E402

n = int(float(sys.argv[1]))
P = int(sys.argv[2])
k = int(sys.argv[sys.argv.index("--k") + 1]) if "--k" in sys.argv else 100
DEV = torch.device("cuda", 0)
g = torch.Generator(device="cuda").manual_seed(1)
p = torch.rand((n, 3), generator=g, device="cuda")
cfg = E.KnnConfig(k=k)

rec: dict = {r: {} for r in range(P)}
_orig_send = PL._halo_send
_orig_publish = PL._publish


def _send(index, radii, comm, cfg_, info, marks=True):
    out = _orig_send(index, radii, comm, cfg_, info, marks)
    rec[comm.rank]["recv"] = out
    return out


def _publish(index, radii, comm, cfg_):
    res = _orig_publish(index, radii, comm, cfg_)
    rec[comm.rank].setdefault("pubs", []).append(res)
    return res


PL._halo_send = _send
PL._publish = _publish


def fn(comm):
    b, e = n * comm.rank // comm.size, n * (comm.rank + 1) // comm.size
    info = PL.RunInfo(PL.PhaseTimer(False, DEV))
    R = PL.redistribute_set(p[b:e], comm, cfg, n)
    rec[comm.rank]["owned"] = R.owned
    rec[comm.rank]["box"] = R.box
    out = PL.compute_set(R, comm, cfg, info)
    rec[comm.rank]["counts"] = dict(info.counts)
    return out


t0 = time.perf_counter()
outs = run_loopback(P, fn, DEV)
torch.cuda.synchronize()
print(f"loopback x{P} {n} (shared GPU): {time.perf_counter() - t0:.2f} s", flush=True)
equal = torch.equal(torch.cat(outs), E.knn_distances(p, k))
print("equal to one rank:", equal, flush=True)
del outs
PL._halo_send, PL._publish = _orig_send, _orig_publish


def timed(fn_):
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    r = fn_()
    b.record()
    b.synchronize()
    return r, a.elapsed_time(b)


rows = []
for r in range(P):
    st = rec[r]
    owned, box = st["owned"], st["box"]
    nr = owned.shape[0]
    hint2 = E.radius_hint(box, n, k)
    index, t_build = timed(lambda: E.build_index(owned, box, grid=True, density_n=n))
    pub_all, depths, offs = st["pubs"][0]  # the published trees (radius bounds) of every rank
    ng = (nr + 63) // 64

    def classify():
        ub = PL._radius_bounds(index, cfg)
        fl = K.boundary_groups(ub, index.depth, ng, pub_all, offs, depths, r)
        return ub, fl, K.compact_flags(fl), K.compact_flags(1 - fl)

    (ub, fl, (blist, bcnt), (ilist, icnt)), t_cls = timed(classify)
    d2 = torch.zeros(nr, dtype=torch.float32, device=DEV)
    fin = torch.empty(nr, dtype=torch.float32, device=DEV)

    def local():
        # as knn_with_halo: both passes queued back to back, their failure checks deferred
        pend: list = []
        E.query(index, cfg, hint2, out=d2, final_out=fin, groups=blist, ngroups=ng, ngroups_dev=bcnt,
                short_list=True, deferred=pend)
        E.query(index, cfg, hint2, out=d2, final_out=fin, groups=ilist, ngroups=ng, ngroups_dev=icnt,
                deferred=pend)
        E.settle(pend)

    _, t_local = timed(local)
    # the two launches apart, and the whole rank in one launch without lists (the kernel's
    # own time at this density: what the split costs)
    _, t_bnd = timed(lambda: E.query(index, cfg, hint2, out=d2, final_out=fin, groups=blist, ngroups=ng,
                                     ngroups_dev=bcnt, short_list=True))
    _, t_int = timed(lambda: E.query(index, cfg, hint2, out=d2, final_out=fin, groups=ilist, ngroups=ng,
                                     ngroups_dev=icnt))
    # the two passes on two streams at once (the interior's workgroups fill the CUs the
    # boundary pass's tail leaves idle); hi: the boundary pass's stream has the high priority
    lo_p, hi_p = torch.cuda.Stream.priority_range()

    def local_conc(hi):
        cur = torch.cuda.current_stream(DEV)
        sa, sb = torch.cuda.Stream(DEV, priority=hi_p if hi else 0), torch.cuda.Stream(DEV)
        sa.wait_stream(cur)
        sb.wait_stream(cur)
        pend: list = []
        with torch.cuda.stream(sa):
            E.query(index, cfg, hint2, out=d2, final_out=fin, groups=blist, ngroups=ng, ngroups_dev=bcnt,
                    short_list=True, deferred=pend)
        with torch.cuda.stream(sb):
            E.query(index, cfg, hint2, out=d2, final_out=fin, groups=ilist, ngroups=ng, ngroups_dev=icnt,
                    deferred=pend)
        cur.wait_stream(sa)
        cur.wait_stream(sb)
        E.settle(pend)

    _, t_conc = timed(lambda: local_conc(False))
    _, t_conc_hi = timed(lambda: local_conc(True))
    d2_all = torch.empty(nr, dtype=torch.float32, device=DEV)
    _, t_all = timed(lambda: E.query(index, cfg, hint2, out=d2_all, final_out=fin))
    del d2_all
    # what this rank sends: its points against the other ranks' exact published radii
    pub2, dep2, off2 = st["pubs"][1]
    mask, t_mask = timed(lambda: K.halo_mask(index.pts[:nr], pub2.reshape(-1), off2, dep2, r))
    recv = st["recv"]
    # (the halo index as the pipeline builds it: with a grid at the local level; timed
    # here, not again inside the re-query — round 5's replay counted it twice)
    hidx, t_htree = timed(lambda: PL.halo_index(index, recv) if recv.shape[0] else None)
    K.tree_set_radii(index.nodes, nr, d2)

    def requery():
        info = PL.RunInfo(PL.PhaseTimer(False, DEV))
        PL._halo_requery(index, d2, recv, cfg, hint2, info, fin, hidx=hidx)
        return info.counts.get("requery_groups", 0)

    if os.environ.get("REPLAY_REQUERY_STATS") and r == 0:
        # (untimed) kernel counters of the re-query: evaluations, passes, backstop
        d2s = d2.clone()
        info = PL.RunInfo(PL.PhaseTimer(False, DEV))
        PL._halo_requery(index, d2s, recv, E.KnnConfig(k=cfg.k, collect_stats=True), hint2, info, fin.clone(),
                         hidx=hidx)
        c = info.stats.counters
        w = max(c.get("waves", 1), 1)
        # flagging + compaction vs the re-query launch (device-synchronised marks, 2nd run)
        tinfo = PL.RunInfo(PL.PhaseTimer(True, DEV))
        tinfo.timer.start()
        PL._halo_requery(index, d2.clone(), recv, cfg, hint2, tinfo, fin.clone(), hidx=hidx)
        print("requery phases ms:", {kk: round(v * 1e3, 2) for kk, v in tinfo.timer.times.items()}, flush=True)
        # the same flagged groups through the local pass alone (one tree, no bound), and
        # as many interior groups: is it the groups or the second source?
        hflags = torch.zeros(ng, dtype=torch.int32, device=DEV)
        K.check(K._native.hip().lsk_hip_flag_groups_inverse(hidx.pts.data_ptr(), hidx.n, index.nodes.data_ptr(),
                                                            index.depth, ng, hflags.data_ptr(),
                                                            K._stream(index.pts)), "flag_groups")
        hl, hc = K.compact_flags(hflags)
        il = ilist[:int(hc.item())].contiguous()
        ic = torch.tensor([il.numel()], dtype=torch.int32, device=DEV)
        dd = d2.clone()
        for nm, gl, gc in (("flagged", hl, hc), ("interior", il, ic)):
            _, tq = timed(lambda: E.query(index, cfg, hint2, out=dd, groups=gl, ngroups=ng, ngroups_dev=gc,
                                          short_list=True))
            print(f"local pass over {int(gc.item())} {nm} groups: {tq:.2f} ms", flush=True)
        print("requery stats:", {kk: c.get(kk, 0) for kk in ("waves", "fallback_queries", "failed_lanes",
                                                             "overflow_lanes", "underflow_lanes")},
              f"evals/w {c.get('evals', 0) / w:.0f} passes/w {c.get('hist_passes', 0) / w:.2f} "
              f"cells/w {c.get('leaves', 0) / w:.1f}", flush=True)
        del d2s

    nreq, t_req = timed(requery)
    res = torch.empty(nr, dtype=torch.float32, device=DEV)
    perm = torch.randperm(nr, device=DEV, dtype=torch.int64).to(torch.int32)
    _, t_ret = timed(lambda: K.scatter1(fin, perm, res, finalize=False))
    row = {"rank": r, "owned": nr, "boundary_groups": int(bcnt.item()), "groups": ng,
           "halo_recv": int(recv.shape[0]), "halo_sent": int((mask != 0).sum()),
           "requery_groups": int(nreq), "build_ms": round(t_build, 2), "classify_ms": round(t_cls, 2),
           "local_ms": round(t_local, 2), "halo_ms": round(t_mask + t_htree, 2), "requery_ms": round(t_req, 2),
           "return_ms": round(t_ret, 2)}
    row["total_ms"] = round(sum(v for kk, v in row.items() if kk.endswith("_ms")), 2)
    row["local_split"] = {"boundary_ms": round(t_bnd, 2), "interior_ms": round(t_int, 2),
                          "one_launch_no_lists_ms": round(t_all, 2), "two_streams_ms": round(t_conc, 2),
                          "two_streams_boundary_hi_ms": round(t_conc_hi, 2)}
    row["grid"] = index.grid.decision() if index.grid is not None else None
    rows.append(row)
    print(json.dumps(row), flush=True)
    del index, hidx, ub, fl, d2, fin, mask, res, perm
    torch.cuda.empty_cache()

summary = {"n": n, "ranks": P, "k": k, "equal_to_one_rank": equal,
           "halo_bytes_total": sum(r_["halo_recv"] for r_ in rows) * 12,
           "max_total_ms": max(r_["total_ms"] for r_ in rows),
           "max": {kk: max(r_[kk] for r_ in rows) for kk in rows[0] if kk.endswith("_ms")},
           "halo_over_local_max": max((r_["halo_ms"] + r_["requery_ms"]) / r_["local_ms"] for r_ in rows)}
print("SUMMARY", json.dumps(summary), flush=True)
