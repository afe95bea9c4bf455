#!/usr/bin/env python3
"""Cell-image-search latency and recall per index tier (reference README: <5 ms Flat, <100 ms
IVFPQ at 58 M vectors, ~95 % recall@10: ``apps/cell-image-search/README.md:130-137``).

Synthetic clustered, L2-normalised 768-d embeddings (random cluster centres + noise) live on the
GPU; for each N the bench builds

* the exact bf16 Flat tier (ground truth),
* the IVF exact-scan tier (list-sorted bf16 slabs in HBM, HIP scan kernel ``be_ivf_scan_bf16``),
  swept over nprobe,
* the IVF-PQ tier (m=96 x 8 bit, the reference's compressed layout) with and without an exact
  re-rank of the PQ shortlist,

and reports p50 / p95 latency of one query and of a 64-query batch (top-20), build time and two
recall figures against the exact ranking: ``recall@10`` = |approx top-10 ∩ exact top-10| / 10
(strict) and ``R@10`` = fraction of queries whose exact nearest neighbour is in the approx top-10
(the FAISS convention the reference's "~95 % recall@10" uses).  One JSON line per (N, tier, nprobe).
Usage: ``python tools/search_bench.py --n 10000000,58000000``
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def synth(n, d, dev, seed=0, chunk=1 << 22):
    """Hierarchical clusters like image embeddings: 4096 class centres (norm 1), 64 sub-centres per
    class (offset norm 0.5), per-vector noise (norm 0.2), L2-normalised."""
    g = torch.Generator(device=dev).manual_seed(seed)
    centres = torch.nn.functional.normalize(torch.randn(4096, d, device=dev, generator=g), dim=1)
    subs = torch.nn.functional.normalize(torch.randn(4096 * 64, d, device=dev, generator=g), dim=1) * 0.5
    out = torch.empty(n, d, dtype=torch.bfloat16, device=dev)
    for i in range(0, n, chunk):
        m = min(chunk, n - i)
        sub = torch.randint(0, 4096 * 64, (m,), device=dev, generator=g)
        v = centres[sub // 64] + subs[sub] + 0.2 * torch.randn(m, d, device=dev, generator=g) / d ** 0.5
        out[i:i + m] = torch.nn.functional.normalize(v, dim=1).bfloat16()
    return out


def ood_queries(nq, d, dev, seed=7):
    """Out-of-distribution queries: the database's class centres (same generator as ``synth``) with
    sub-centre offsets that were NEVER used for indexed vectors, plus noise -- the nearest neighbours
    are spread over the class instead of sitting next to the query, unlike indexed-vector + noise."""
    g = torch.Generator(device=dev).manual_seed(0)
    centres = torch.nn.functional.normalize(torch.randn(4096, d, device=dev, generator=g), dim=1)
    gq = torch.Generator(device=dev).manual_seed(seed + 1000)
    cls = torch.randint(0, 4096, (nq,), device=dev, generator=gq)
    held_out = torch.nn.functional.normalize(torch.randn(nq, d, device=dev, generator=gq), dim=1) * 0.5
    v = centres[cls] + held_out + 0.2 * torch.randn(nq, d, device=dev, generator=gq) / d ** 0.5
    return torch.nn.functional.normalize(v, dim=1)


def timeit(fn, reps):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
    ts.sort()
    return ts[len(ts) // 2], ts[int(0.95 * (len(ts) - 1))]


def recalls(gt, got):
    r10 = float(np.mean([len(set(g[:10]) & set(r[:10])) / 10 for g, r in zip(gt, got)]))
    r1 = float(np.mean([g[0] in set(r[:10]) for g, r in zip(gt, got)]))
    return round(r10, 4), round(r1, 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="1000000,10000000")
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--nprobes", default="16,32,64,128,256")
    ap.add_argument("--no-pq", action="store_true")
    ap.add_argument("--tiers", default="ivf,pq96,compressed",
                    help="ivf: exact-scan IVF; pq96: IVF-PQ m=96 (+ GPU re-rank); compressed: IVF-PQ m=192 on "
                         "the GPU with the full vectors in host memory as the re-rank store (VectorIndex.compress)")
    ap.add_argument("--refines", default="400,1000,2000", help="compressed tier: re-ranked candidates per query")
    ap.add_argument("--queries", default="near,ood", help="near: indexed vectors + small noise; "
                    "ood: held-out sub-centres of the indexed classes (ood_queries)")
    a = ap.parse_args()
    from bioengine_worker_amd.search.index import VectorIndex
    from bioengine_worker_amd.search.ivfpq import IVFPQIndex, default_nlist

    dev = torch.device("cuda", 0)
    for n in [int(v) for v in a.n.split(",")]:
        x = synth(n, a.dim, dev)
        gq = torch.Generator(device=dev).manual_seed(7)
        qidx = torch.randint(0, n, (64,), device=dev, generator=gq)
        qsets = {"near": torch.nn.functional.normalize(
            x[qidx].float() + 0.02 * torch.randn(64, a.dim, device=dev, generator=gq), dim=1),
            "ood": ood_queries(64, a.dim, dev)}
        qsets = {k: v for k, v in qsets.items() if k in a.queries.split(",")}
        flat = VectorIndex(dim=a.dim, device=dev, index_type="flat")
        flat.vecs = x
        # ground truth in fp32 (fp32 query x bf16 vectors upcast per chunk): exact up to fp32 rounding
        gts = {}
        for qn, qv in qsets.items():
            gs, gi = [], []
            for i in range(0, n, 1 << 20):
                sc = qv @ x[i:i + (1 << 20)].float().T
                ts, ti = torch.topk(sc, a.k, dim=1)
                gs.append(ts)
                gi.append(ti + i)
            ts, j = torch.topk(torch.cat(gs, 1), a.k, dim=1)
            gts[qn] = torch.gather(torch.cat(gi, 1), 1, j).cpu().numpy()
        q = next(iter(qsets.values()))
        for name, fn in (("flat_q1", lambda: flat.search(q[:1], a.k)), ("flat_q64", lambda: flat.search(q, a.k))):
            fn()
            p50, p95 = timeit(fn, a.reps)
            print(json.dumps({"n": n, "tier": "FlatIP-GPU bf16", "query": name, "p50_ms": round(p50, 3),
                              "p95_ms": round(p95, 3), "recall@10": 1.0, "R@10": 1.0}), flush=True)
        tiers = a.tiers.split(",")
        # ---- IVF exact scan over list-sorted HBM slabs
        t0 = time.perf_counter()
        ivf = VectorIndex(dim=a.dim, device=dev, index_type="ivf")
        ivf.vecs = x
        if "ivf" in tiers:
            ivf.train_ivf()
        nprobes = [int(v) for v in a.nprobes.split(",")] if "ivf" in tiers else []
        torch.cuda.synchronize()
        build = time.perf_counter() - t0
        nl = ivf.centroids.shape[0] if ivf.centroids is not None else 0
        for npb in nprobes:
            rec = {qn: recalls(gts[qn], ivf.search(qv, a.k, nprobe=npb)[1]) for qn, qv in qsets.items()}
            r10, r1 = next(iter(rec.values()))
            for name, qq in (("q1", q[:1]), ("q64", q)):
                ivf.search(qq, a.k, nprobe=npb)
                p50, p95 = timeit(lambda: ivf.search(qq, a.k, nprobe=npb), a.reps)
                print(json.dumps({"n": n, "tier": "IVF-exact-scan bf16 (HBM)", "nprobe": npb, "nlist": nl, "query": name,
                                  "p50_ms": round(p50, 3), "p95_ms": round(p95, 3), "recall@10": r10, "R@10": r1,
                                  "recall@10_by_queries": {k: v[0] for k, v in rec.items()},
                                  "R@10_by_queries": {k: v[1] for k, v in rec.items()},
                                  "build_s": round(build, 2), "hbm_gb": round(2 * x.numel() * 2 / 1e9, 2)}), flush=True)
        del ivf
        torch.cuda.empty_cache()
        if a.no_pq:
            del x, flat
            torch.cuda.empty_cache()
            continue
        if "compressed" in tiers:
            # ---- compressed tier: m=192 PQ codes on the GPU, full vectors in host memory (re-rank store)
            print(json.dumps({"n": n, "stage": "compressed tier build (IVF-PQ m=192 + host copy)"}), flush=True)
            t0 = time.perf_counter()
            cvi = VectorIndex(dim=a.dim, device=dev, index_type="ivfpq")
            cvi.vecs = x
            fp = cvi.compress(pq_m=192, refine=50)
            torch.cuda.synchronize()
            build = time.perf_counter() - t0
            for R in [int(v) for v in a.refines.split(",")]:
                cvi.refine = max(1, R // a.k)
                rec = {qn: recalls(gts[qn], cvi.search(qv, a.k)[1]) for qn, qv in qsets.items()}
                r10, r1 = next(iter(rec.values()))
                for name, qq in (("q1", q[:1]), ("q64", q)):
                    cvi.search(qq, a.k)
                    p50, p95 = timeit(lambda: cvi.search(qq, a.k), max(3, a.reps // 2))
                    print(json.dumps({"n": n, "tier": f"IVFPQ m=192 GPU + host re-rank {cvi.refine * a.k}",
                                      "query": name, "p50_ms": round(p50, 3), "p95_ms": round(p95, 3),
                                      "recall@10": r10, "R@10": r1,
                                      "recall@10_by_queries": {k: v[0] for k, v in rec.items()},
                                      "R@10_by_queries": {k: v[1] for k, v in rec.items()},
                                      "nlist": cvi.pq.nlist, "nprobe": cvi.pq.nprobe, "build_s": round(build, 2),
                                      "gpu_index_gb": round(fp["gpu_bytes"] / 1e9, 3),
                                      "host_refine_gb": round(fp["host_bytes"] / 1e9, 3)}), flush=True)
            del cvi
            torch.cuda.empty_cache()
        if "pq96" not in tiers:
            del x, flat
            torch.cuda.empty_cache()
            continue
        # ---- IVF-PQ (the reference's compressed layout), PQ-only and with exact re-rank
        t0 = time.perf_counter()
        npl = default_nlist(n)
        pq = IVFPQIndex(dim=a.dim, nlist=npl, m=96, nprobe=64, device=dev)
        pq.train(x.float() if n <= 2_000_000 else x[torch.randperm(n, device=dev)[:2_000_000]].float())
        pq.add(x)
        torch.cuda.synchronize()
        build = time.perf_counter() - t0
        for refine, tier in ((0, "IVFPQ-GPU m=96 nprobe=64"), (4, "IVFPQ-GPU + exact rerank 80"),
                             (200, "IVFPQ-GPU + exact rerank 4k")):
            vi = VectorIndex(dim=a.dim, device=dev, index_type="ivfpq", refine=refine)
            vi.vecs, vi.pq = x, pq
            rec = {qn: recalls(gts[qn], vi.search(qv, a.k)[1]) for qn, qv in qsets.items()}
            r10, r1 = next(iter(rec.values()))
            for name, qq in (("q1", q[:1]), ("q64", q)):
                vi.search(qq, a.k)
                p50, p95 = timeit(lambda: vi.search(qq, a.k), a.reps)
                print(json.dumps({"n": n, "tier": tier, "query": name, "p50_ms": round(p50, 3), "p95_ms": round(p95, 3),
                                  "recall@10": r10, "R@10": r1, "recall@10_by_queries": {k: v[0] for k, v in rec.items()},
                                  "R@10_by_queries": {k: v[1] for k, v in rec.items()},
                                  "nlist": pq.nlist, "build_s": round(build, 2),
                                  "codes_gb": round(pq.codes.numel() / 1e9, 3)}), flush=True)
        del x, flat, pq, vi
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
