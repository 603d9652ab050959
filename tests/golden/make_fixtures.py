"""Generate the committed golden fixtures from the REFERENCE's own client code.

Run in the build container only (it needs /root/reference):
    python tests/golden/make_fixtures.py [--wire-only | --client-only]

What it imports from the reference (read-only, never copied):
  src/utils.py  : zero_except_top_k_weights, serialize_sparse, serialize_dense,
                  encrypt_parameters, flatten_params, get_learnable_parameters
  src/update.py : l2clipping, diff_weights
  src/models.py : MLP (MLP-MNIST, d = 50,890)
  src/secure_aggregation_pb2.py : the generated proto messages (wire.npz: request /
                  response bytes as the reference's client serialises them; importable
                  only with the pure-Python protobuf backend)
utils.py loads 'src/libsgx_enc.so' relative to the cwd at import time.  The
prebuilt binary shipped in the reference is NEVER loaded: we run from a scratch
cwd whose src/libsgx_enc.so is oracle/_ref/libsgx_enc.so, compiled by
oracle/Makefile from the reference's own src/cpp/encryption.cpp.
torchvision is absent here, so a stub module is injected (utils.py only uses it
for dataset loaders, which are out of scope).

Outputs (tests/golden/*.npz) hold inputs and the reference-produced bytes
(plaintext records, ciphertext), plus the oracle's aggregates at generation
time for regression.  ref_aggregate.npz pins the aggregation arithmetic itself:
its expected aggregates are the output of the reference's own in-order
aggregator, src/update.py:173-184 update_global_weights (the fl_main.py:251-253
path), run here on the same client updates whose payloads it stores (the Rust
enclave cannot run here; this is the reference code that computes the same
per-index in-order fp32 sum).
"""
import os

# the reference's old generated pb2 needs the pure-Python protobuf backend; the
# backend is fixed at the first protobuf import, so set it before anything else
os.environ.setdefault("PROTOCOL_BUFFERS_PYTHON_IMPLEMENTATION", "python")
import shutil
import sys
import tempfile
import types

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF_SRC = "/root/reference/src"
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle as O  # noqa: E402


def import_reference():
    O.build()
    assert os.path.exists(O.REF_AES_PATH), "oracle/_ref/libsgx_enc.so missing"
    scratch = tempfile.mkdtemp(prefix="fltee_fix_")
    os.makedirs(os.path.join(scratch, "src"))
    shutil.copy(O.REF_AES_PATH, os.path.join(scratch, "src", "libsgx_enc.so"))
    tv = types.ModuleType("torchvision")
    tv.datasets = types.SimpleNamespace()
    tv.transforms = types.SimpleNamespace()
    sys.modules["torchvision"] = tv
    sys.path.insert(0, REF_SRC)
    cwd = os.getcwd()
    os.chdir(scratch)
    try:
        import models
        import update
        import utils
    finally:
        os.chdir(cwd)
    return utils, update, models


def perturbed_diff(model, seed, scale=0.01):
    g = torch.Generator().manual_seed(seed)
    diff = {}
    for key, val in model.state_dict().items():
        diff[key] = torch.randn(val.shape, generator=g) * scale
    from collections import OrderedDict
    return OrderedDict(diff)


def wire_fixtures():
    """proto/secure_aggregation.proto messages serialised by the reference's pb2."""
    sys.path.insert(0, REF_SRC)
    import secure_aggregation_pb2 as pb
    sp = np.load(os.path.join(OUT, "mnist_sparse.npz"))
    ids = sp["client_ids"].astype(np.uint32)
    d, k = int(sp["d"]), int(sp["k"])
    upd = sp["oracle_advanced"].astype(np.float32)
    start_req = dict(fl_id=0, client_ids=list(range(100)), sigma=1.12, clipping=1.0, alpha=0.1,
                     sampling_ratio=0.3, aggregation_alg=1, num_of_parameters=d,
                     num_of_sparse_parameters=k)
    start_resp = dict(fl_id=0, round=0, client_ids=[int(x) for x in ids])
    agg_req = dict(fl_id=0, round=0, encrypted_parameters=sp["ciphertext"].tobytes(),
                   num_of_parameters=d, num_of_sparse_parameters=k, optimal_num_of_clients=100,
                   aggregation_alg=1, client_ids=[int(x) for x in ids])
    agg_resp = dict(updated_parameters=upd.tolist(), execution_time=0.125,
                    client_ids=[int(x) for x in ids[::-1]], round=1)
    big_ids = dict(fl_id=4294967295, round=70000, client_ids=[0, 127, 128, 16383, 16384, 4294967295])
    out = {}
    for name, cls, fields in [("start_req", pb.StartRequestParameters, start_req),
                              ("start_resp", pb.StartResponseParameters, start_resp),
                              ("agg_req", pb.AggregateRequestParameters, agg_req),
                              ("agg_resp", pb.AggregateResponseParameters, agg_resp),
                              ("start_resp_edge", pb.StartResponseParameters, big_ids),
                              ("agg_req_empty", pb.AggregateRequestParameters, {})]:
        out[name] = np.frombuffer(cls(**fields).SerializeToString(), dtype=np.uint8)
    np.savez_compressed(os.path.join(OUT, "wire.npz"), **out, start_sigma=np.float32(1.12),
                        start_clipping=np.float32(1.0), start_alpha=np.float32(0.1),
                        start_ratio=np.float32(0.3), d=d, k=k, client_ids=ids, updated=upd,
                        ciphertext=sp["ciphertext"], edge_ids=np.array(big_ids["client_ids"],
                                                                        dtype=np.uint64))
    print("wire", {k_: v.size for k_, v in out.items()})


def client_fixtures(utils, update, models):
    """The client producers of fl_main.py:221-238 run by the reference's own functions
    on explicit flat updates (stored, so the GPU test needs no reference import).
    Clients 2 and 3 are quantised to multiples of 1e-3: heavy |val| ties exercise the
    stable-sort tie order of zero_except_top_k_weights."""
    from collections import OrderedDict
    model = models.MLP(dim_in=784, dim_hidden=64, dim_out=10)
    bn = utils.get_buffer_names(model)
    d = utils.count_parameters(model)
    k = int(0.1 * d)
    ids = np.array([5, 77, 1234, 65535], dtype=np.uint32)
    g = torch.Generator().manual_seed(4242)
    flats = torch.randn(len(ids), d, generator=g) * 0.01
    flats[2:] = torch.round(flats[2:] * 1000) / 1000
    flats[3, :50] = 0.0
    flats[3, 50:60] = -0.0

    def as_state(flat):
        st, off = OrderedDict(), 0
        for key, val in model.state_dict().items():
            st[key] = flat[off:off + val.numel()].reshape(val.shape).clone()
            off += val.numel()
        return st

    topk, plain, plain_clip, cipher, dense_plain, dense_clip = [], [], [], [], [], []
    for cid, flat in zip(ids, flats):
        st = as_state(flat)
        top, idxs = utils.zero_except_top_k_weights(st, bn, k)
        topk.append(np.asarray(idxs, np.uint32))
        b = utils.serialize_sparse(top, bn, idxs)
        plain.append(np.frombuffer(b, np.uint8))
        cipher.append(np.frombuffer(bytes(utils.encrypt_parameters(b, int(cid))), np.uint8))
        bc = utils.serialize_sparse(update.l2clipping(top, bn, 1.0), bn, idxs)
        plain_clip.append(np.frombuffer(bc, np.uint8))
        dense_plain.append(np.frombuffer(utils.serialize_dense(st, bn, d), np.uint8))
        dense_clip.append(np.frombuffer(utils.serialize_dense(update.l2clipping(st, bn, 0.05), bn, d),
                                        np.uint8))
    np.savez_compressed(os.path.join(OUT, "client_producer.npz"), client_ids=ids,
                        flats=flats.numpy().astype(np.float32), d=d, k=k, topk=np.stack(topk),
                        plain=np.concatenate(plain), plain_clip=np.concatenate(plain_clip),
                        cipher=np.concatenate(cipher), dense_plain=np.concatenate(dense_plain),
                        dense_clip=np.concatenate(dense_clip), clipping=1.0, dense_clipping=0.05)
    print("client_producer d", d, "k", k)


REF_AGG_CASES = [  # (name, model, dense, n): n power of two -> torch.div == x * (1/n)
    ("sparse_n4", "mnist", False, 4),
    ("sparse_n32", "mnist", False, 32),
    ("sparse_n30", "mnist", False, 30),
    ("sparse_n100", "mnist", False, 100),
    ("dense_n4", "small", True, 4),
    ("dense_n30", "small", True, 30),
    ("dense_n32", "small", True, 32),
]


def reference_aggregate_fixtures(utils, update, models):
    """The reference's OWN aggregate on the same client updates.

    src/update.py:173-184 update_global_weights is the fl_main.py:251-253 in-order
    aggregator: w_avg = diffs[0]; w_avg += diffs[i] for i = 1..n-1 (client order);
    torch.div(w_avg, n); global += w_avg.  Run here on a zero global model it returns
    the averaged update.  The sparse cases feed it the top-k-zeroed state dicts that
    zero_except_top_k_weights returns (utils.py:327-354), the dense cases the full
    diffs; the payload of each client is serialize_sparse / serialize_dense of the
    same state (fl_main.py:221-238), in the same client order.

    The enclave sums the same values per index in the same order from +0.0 and
    multiplies by 1f32/n (common.rs:14-19); torch.div divides.  For a power-of-two n
    the two are the same IEEE operation (bit-exact); otherwise they differ by at most
    one ulp.  Stored per case: client_ids, plaintext records (the reference's bytes),
    d, k, ref_avg (update_global_weights' output, flattened) and abs_sum (sum of
    |client values| per index, f64, for the reassociation bound of advanced/nips19).
    Ciphertexts are not stored: tests encrypt with the oracle's AES, which is pinned to
    the reference's encryption.cpp (test_oracle.py)."""
    from collections import OrderedDict
    out = {}
    for name, which, dense, n in REF_AGG_CASES:
        if which == "mnist":
            model = models.MLP(dim_in=784, dim_hidden=64, dim_out=10)  # d = 50,890
        else:  # a small MLP for the dense payloads (d = 3,562) to keep fixtures small
            model = models.MLP(dim_in=100, dim_hidden=32, dim_out=10)
        bn = utils.get_buffer_names(model)
        d = utils.count_parameters(model)
        k = d if dense else int(0.1 * d)
        ids = (np.arange(n, dtype=np.uint32) * 7 + 11).astype(np.uint32)
        states, plain = [], []
        for cid in ids:
            diff = perturbed_diff(model, seed=5000 + int(cid) + 100000 * n)
            if dense:
                st = diff
                b = utils.serialize_dense(st, bn, d)
            else:
                st, idxs = utils.zero_except_top_k_weights(diff, bn, k)
                b = utils.serialize_sparse(st, bn, idxs)
            states.append(OrderedDict((key, v.clone()) for key, v in st.items()))
            plain.append(np.frombuffer(b, np.uint8))
        flats = [utils.flatten_params(utils.get_learnable_parameters(s, bn)).numpy().astype(np.float64)
                 for s in states]
        abs_sum = np.sum(np.abs(np.stack(flats)), axis=0)
        glob = OrderedDict((key, torch.zeros_like(v)) for key, v in model.state_dict().items())
        update.update_global_weights(glob, states)   # the reference's aggregator
        ref_avg = utils.flatten_params(utils.get_learnable_parameters(glob, bn)).numpy()
        out[name] = dict(client_ids=ids, plaintext=np.concatenate(plain), d=d, k=k, n=n,
                         dense=dense, ref_avg=ref_avg.astype(np.float32),
                         abs_sum=abs_sum.astype(np.float32))
        print("ref_aggregate", name, "d", d, "k", k, "n", n)
    flat = {}
    for name, fx in out.items():
        for key, v in fx.items():
            flat[name + "__" + key] = np.asarray(v)
    flat["cases"] = np.array([c[0] for c in REF_AGG_CASES])
    np.savez_compressed(os.path.join(OUT, "ref_aggregate.npz"), **flat)


CFG_CASES = [  # (name, dense, n): BASELINE configs[3]'s shape, Purchase100 x 300 clients
    ("purchase100_sparse_n300", False, 300),
    ("purchase100_dense_n300", True, 300),
]


def config_aggregate_fixtures(utils, update, models):
    """The reference's own aggregate at a benchmark configuration's full size
    (ref_aggregate_cfg.npz): MLPPurchase100 (fl_main.py:69-77, d = 44,964), 300 clients,
    alpha = 0.1 top-k (k = 4,496) and dense — configs[3]'s shape.

    The 300 payloads (10.8 MB sparse, 108 MB dense) are not stored.  They are a pure
    function of the stored seeds and parameter shapes: each client's diff is
    perturbed_diff (torch.randn from its seed, in state-dict order), its payload
    zero_except_top_k_weights + serialize_sparse (utils.py:327-354,193-209: stable sort
    by |value| descending, the first k) or serialize_dense.  tests/refcheck.py
    regenerates the records with numpy/torch and checks them against the sha256 of the
    reference's bytes stored here, so the expected aggregate (update_global_weights,
    update.py:173-184) is pinned to the reference's own client and aggregator code."""
    import hashlib
    from collections import OrderedDict
    model = models.MLPPurchase100(dim_in=600, dim_hidden=64, dim_out=100)
    bn = utils.get_buffer_names(model)
    d = utils.count_parameters(model)
    shapes = [tuple(v.shape) for key, v in model.state_dict().items() if key not in bn]
    flat = {}
    for ci, (name, dense, n) in enumerate(CFG_CASES):
        k = d if dense else int(0.1 * d)
        ids = (np.arange(n, dtype=np.uint32) * 7 + 11).astype(np.uint32)
        seeds = (np.arange(n, dtype=np.int64) + 900_000 + 10_000 * ci).astype(np.int64)
        h = hashlib.sha256()
        states = []
        for seed in seeds:
            diff = perturbed_diff(model, seed=int(seed))
            if dense:
                st = diff
                b = utils.serialize_dense(st, bn, d)
            else:
                st, idxs = utils.zero_except_top_k_weights(diff, bn, k)
                b = utils.serialize_sparse(st, bn, idxs)
            h.update(b)
            states.append(OrderedDict((key, v.clone()) for key, v in st.items()))
        glob = OrderedDict((key, torch.zeros_like(v)) for key, v in model.state_dict().items())
        update.update_global_weights(glob, states)   # the reference's aggregator
        ref_avg = utils.flatten_params(utils.get_learnable_parameters(glob, bn)).numpy()
        fx = dict(client_ids=ids, seeds=seeds, d=d, k=k, n=n, dense=dense,
                  ref_avg=ref_avg.astype(np.float32), payload_sha256=h.hexdigest(),
                  scale=0.01)
        for key, v in fx.items():
            flat[name + "__" + key] = np.asarray(v)
        print("ref_aggregate_cfg", name, "d", d, "k", k, "n", n, h.hexdigest()[:16])
    flat["cases"] = np.array([c[0] for c in CFG_CASES])
    flat["shapes"] = np.array([list(s) + [1] * (2 - len(s)) for s in shapes], dtype=np.int64)
    flat["shape_rank"] = np.array([len(s) for s in shapes], dtype=np.int64)
    np.savez_compressed(os.path.join(OUT, "ref_aggregate_cfg.npz"), **flat)


def main():
    if "--wire-only" in sys.argv:
        wire_fixtures()
        return
    utils, update, models = import_reference()
    if "--client-only" in sys.argv:
        client_fixtures(utils, update, models)
        return
    if "--ref-aggregate-only" in sys.argv:
        reference_aggregate_fixtures(utils, update, models)
        return
    if "--ref-aggregate-cfg-only" in sys.argv:
        config_aggregate_fixtures(utils, update, models)
        return
    torch.manual_seed(1)

    # ---------------- MLP-MNIST sparse (alpha = 0.1), fl_main.py:221-238 ----------
    model = models.MLP(dim_in=784, dim_hidden=64, dim_out=10)
    buffer_names = utils.get_buffer_names(model)
    d = utils.count_parameters(model)
    alpha = 0.1
    k = int(alpha * d)
    client_ids = np.array([3, 17, 42, 99], dtype=np.uint32)
    for clip in (False, True):
        plain, enc, topk = [], [], []
        for cid in client_ids:
            diff = perturbed_diff(model, seed=1000 + int(cid))
            top, idxs = utils.zero_except_top_k_weights(diff, buffer_names, k)
            if clip:
                top = update.l2clipping(top, buffer_names, 1.0)
            b = utils.serialize_sparse(top, buffer_names, idxs)
            e = bytes(utils.encrypt_parameters(b, int(cid)))
            plain.append(np.frombuffer(b, dtype=np.uint8))
            enc.append(np.frombuffer(e, dtype=np.uint8))
            topk.append(np.asarray(idxs, dtype=np.uint32))
        plain = np.concatenate(plain)
        enc = np.concatenate(enc)
        w = O.decrypt_and_parse(client_ids, enc)
        n = len(client_ids)
        g_non, _ = O.non_oblivious(w, d, n)
        g_adv, _ = O.advanced(k, w, d, n)
        name = "mnist_sparse_clip" if clip else "mnist_sparse"
        np.savez_compressed(os.path.join(OUT, name + ".npz"), client_ids=client_ids,
                            plaintext=plain, ciphertext=enc, topk=np.stack(topk), d=d, k=k,
                            alpha=alpha, oracle_non_oblivious=g_non, oracle_advanced=g_adv)
        print(name, "d", d, "k", k, "bytes", enc.nbytes)

    # ---------------- dense uploads (no --alpha): serialize_dense ---------------
    small = torch.nn.Sequential(torch.nn.Linear(20, 10), torch.nn.ReLU(), torch.nn.Linear(10, 5))
    bn = utils.get_buffer_names(small)
    d2 = utils.count_parameters(small)
    ids2 = np.array([0, 1, 7], dtype=np.uint32)
    plain, enc = [], []
    for cid in ids2:
        diff = perturbed_diff(small, seed=2000 + int(cid))
        b = utils.serialize_dense(diff, bn, d2)
        e = bytes(utils.encrypt_parameters(b, int(cid)))
        plain.append(np.frombuffer(b, dtype=np.uint8))
        enc.append(np.frombuffer(e, dtype=np.uint8))
    plain = np.concatenate(plain)
    enc = np.concatenate(enc)
    w = O.decrypt_and_parse(ids2, enc)
    g_base = O.baseline(w, d2, len(ids2))
    np.savez_compressed(os.path.join(OUT, "dense_small.npz"), client_ids=ids2, plaintext=plain,
                        ciphertext=enc, d=d2, oracle_baseline=g_base)
    print("dense_small d", d2)

    # ---------------- l2clipping (update.py:187-204) on a full state dict -------
    diff = perturbed_diff(model, seed=77, scale=0.05)
    clipped = update.l2clipping(diff, buffer_names, 1.0)
    flat_in = utils.flatten_params(utils.get_learnable_parameters(diff, buffer_names)).numpy()
    flat_out = utils.flatten_params(utils.get_learnable_parameters(clipped, buffer_names)).numpy()
    np.savez_compressed(os.path.join(OUT, "l2clip.npz"), flat_in=flat_in.astype(np.float32),
                        flat_out=flat_out.astype(np.float32), clipping=1.0)
    print("l2clip d", flat_in.size)

    # ---------------- client_level_dp_update_global_weights (update.py:207-224) --
    # zero diffs: global += (0 + N(0, C*sigma)) / n, numpy RandomState(seed + 5)
    # (fl_main.py:49) — the reference's seeded DP noise, for distribution checks
    import numpy.random as npr
    n_dp, sigma, clipping = 30, 1.12, 1.0
    zeros = {key: torch.zeros_like(v) for key, v in model.state_dict().items()}
    glob = {key: torch.zeros_like(v) for key, v in model.state_dict().items()}
    update.client_level_dp_update_global_weights(glob, [zeros] * n_dp, sigma, clipping, 0.1,
                                                 npr.RandomState(0 + 5))
    dp_flat = utils.flatten_params(utils.get_learnable_parameters(glob, buffer_names)).numpy()
    np.savez_compressed(os.path.join(OUT, "dp_reference.npz"), noise=dp_flat.astype(np.float32),
                        n=n_dp, sigma=sigma, clipping=clipping)
    print("dp_reference d", dp_flat.size, "std", dp_flat.std())

    # ---------------- src/ffi_test.py known answer (100 x 0x01, key 0, IV 0) ----
    src = bytes([1] * 100)
    ct = O.ref_aes_ctr_encrypt(bytes(16), src)
    np.savez_compressed(os.path.join(OUT, "ffi_test_kat.npz"), plaintext=np.frombuffer(src, np.uint8),
                        ciphertext=np.frombuffer(ct, np.uint8))
    print("ffi kat ok")
    client_fixtures(utils, update, models)
    reference_aggregate_fixtures(utils, update, models)
    config_aggregate_fixtures(utils, update, models)
    wire_fixtures()


if __name__ == "__main__":
    main()
