"""Comparisons against the reference's own aggregate (tests/golden/ref_aggregate.npz).

The fixture's ref_avg is src/update.py:173-184 update_global_weights run on the
clients' updates: the per-index fp32 sum in client order, then torch.div(., n).
The enclave (and this build) sums the same values from +0.0 and multiplies by
1f32/n (common.rs:14-19).  Criteria:

* in-order algorithms (non_oblivious, baseline, path_oram; alg 6 with batch = n):
  bit-exact for power-of-two n (division by n == multiplication by 1/n), at most
  1 ulp otherwise;
* reassociating algorithms (advanced's sort order, nips19's shuffled order, alg 6
  batches): the north-star criterion, 1e-6 relative (norm-wise over the vector),
  plus the per-index reassociation bound 2(n-1)u*sum|x|/n + 2u|ref| (u = 2^-24).
"""
import os

import numpy as np

from conftest import GOLDEN

U = 2.0 ** -24
_cache = {}


def cases():
    fx = _load()
    return [str(c) for c in fx["cases"]]


def _load():
    if "fx" not in _cache:
        _cache["fx"] = np.load(os.path.join(GOLDEN, "ref_aggregate.npz"))
    return _cache["fx"]


def case(name):
    fx = _load()
    c = {key: fx[name + "__" + key] for key in
         ("client_ids", "plaintext", "d", "k", "n", "dense", "ref_avg", "abs_sum")}
    c["d"], c["k"], c["n"] = int(c["d"]), int(c["k"]), int(c["n"])
    c["dense"] = bool(c["dense"])
    c["name"] = name
    return c


def ordered_bits(a):
    """float32 -> integers whose difference is the ulp distance (+0 == -0)."""
    u = np.asarray(a, np.float32).view(np.uint32).astype(np.int64)
    return np.where(u >= 2 ** 31, -(u - 2 ** 31), u)


def ulp_distance(a, b):
    return np.abs(ordered_bits(a) - ordered_bits(b))


def is_pow2(n):
    return n > 0 and (n & (n - 1)) == 0


def assert_in_order_exact(out, c):
    """out vs update_global_weights: bit-exact at power-of-two n, else <= 1 ulp."""
    ulp = ulp_distance(out, c["ref_avg"])
    worst = int(ulp.max()) if ulp.size else 0
    if is_pow2(c["n"]):
        assert worst == 0, f"{c['name']}: {int((ulp > 0).sum())} indices differ (max {worst} ulp)"
    else:
        assert worst <= 1, f"{c['name']}: max {worst} ulp"
    return worst


def assert_reassociated(out, c, rel=1e-6):
    """out vs update_global_weights for an order-changing algorithm."""
    ref = c["ref_avg"].astype(np.float64)
    o = np.asarray(out, np.float32).astype(np.float64)
    assert np.isfinite(o).all()
    n = c["n"]
    norm_rel = np.linalg.norm(o - ref) / max(np.linalg.norm(ref), 1e-300)
    assert norm_rel <= rel, f"{c['name']}: norm-wise relative error {norm_rel:.3e} > {rel}"
    bound = 2 * (n - 1) * U * c["abs_sum"].astype(np.float64) / n + 2 * U * np.abs(ref) + 1e-45
    excess = np.abs(o - ref) - bound
    assert (excess <= 0).all(), f"{c['name']}: {int((excess > 0).sum())} indices over the bound"
    return norm_rel


def records(c):
    """The reference's plaintext payload as oracle.WEIGHT records (client-major)."""
    import oracle as O
    if "recs" in c:
        return c["recs"]
    return np.frombuffer(c["plaintext"].tobytes(), dtype=O.WEIGHT)


# ---- configuration-size cases (ref_aggregate_cfg.npz, make_fixtures.py
# config_aggregate_fixtures): the payloads are regenerated from the stored seeds and
# checked against the sha256 of the bytes the reference's client code produced


def _load_cfg():
    if "cfg" not in _cache:
        _cache["cfg"] = np.load(os.path.join(GOLDEN, "ref_aggregate_cfg.npz"))
    return _cache["cfg"]


def cfg_cases():
    return [str(c) for c in _load_cfg()["cases"]]


def regen_records(shapes, seeds, k, dense, scale=0.01):
    """Each client's diff as make_fixtures.perturbed_diff draws it (torch.randn from the
    seed, parameter by parameter), flattened; its payload as the reference's
    zero_except_top_k_weights + serialize_sparse build it (utils.py:327-354,193-209:
    a stable sort by |value| descending, the first k, in that order) or serialize_dense
    (every index in order)."""
    import torch

    import oracle as O
    out = []
    for s in seeds:
        g = torch.Generator().manual_seed(int(s))
        flat = torch.cat([(torch.randn(sh, generator=g) * scale).reshape(-1) for sh in shapes]).numpy()
        idx = (np.arange(flat.size) if dense else np.argsort(-np.abs(flat), kind="stable")[:k])
        w = np.empty(idx.size, dtype=O.WEIGHT)
        w["idx"] = idx
        w["val"] = flat[idx]
        out.append(w)
    return np.concatenate(out)


def cfg_case(name):
    import hashlib
    if ("cfgcase", name) in _cache:
        return _cache[("cfgcase", name)]
    fx = _load_cfg()
    rank = fx["shape_rank"]
    shapes = [tuple(int(x) for x in s[:r]) for s, r in zip(fx["shapes"], rank)]
    c = {key: fx[name + "__" + key] for key in ("client_ids", "seeds", "d", "k", "n", "dense",
                                                 "ref_avg", "payload_sha256", "scale")}
    c["d"], c["k"], c["n"] = int(c["d"]), int(c["k"]), int(c["n"])
    c["dense"] = bool(c["dense"])
    c["name"] = name
    recs = regen_records(shapes, c["seeds"], c["k"], c["dense"], float(c["scale"]))
    assert hashlib.sha256(recs.tobytes()).hexdigest() == str(c["payload_sha256"]), \
        f"{name}: regenerated payload differs from the reference client's bytes"
    c["recs"] = recs
    vals = recs["val"].astype(np.float64)
    c["abs_sum"] = np.bincount(recs["idx"], weights=np.abs(vals), minlength=c["d"])
    _cache[("cfgcase", name)] = c
    return c
