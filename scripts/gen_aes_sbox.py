#!/usr/bin/env python3
"""Generate fl-tee_amd/csrc/aes_sbox_bs.h: a constant-time, bitsliced AES S-box circuit.

The enclave decrypts with sgx_tcrypto (AES-NI: no secret-dependent addresses,
lib.rs:312-343).  The GPU kernel in k_aes.hip therefore evaluates the S-box as a
boolean circuit on bit planes (one bit of 32 blocks per 32-bit word) instead of table
lookups.  The circuit is the GF(2^8) inverse in a tower field GF(((2^2)^2)^2)
(polynomial bases, Karatsuba products: 36 ANDs), between two 8x8 GF(2) basis changes;
the output change includes FIPS-197's affine matrix, and the affine constant 0x63 is
left out (the kernel folds it into the round keys: ShiftRows/MixColumns map the
all-0x63 state to itself).  Linear layers are materialised with Paar's greedy
common-subexpression heuristic, and the tower (the GF(16) and GF(256) extension
constants mu, lambda and the image beta of the AES generator x) is chosen by
exhaustive search for the fewest XORs.

The script checks the circuit on all 256 inputs (truth tables as 256-bit integers)
against the S-box computed from its definition (FIPS-197 §5.1.1) before writing.
"""
import itertools
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "fl-tee_amd", "csrc", "aes_sbox_bs.h")


# ---------------------------------------------------------------- GF(2^8), AES basis
def gmul(a, b, poly=0x11B, deg=8):
    p = 0
    while b:
        if b & 1:
            p ^= a
        a <<= 1
        if a >> deg:
            a ^= poly
        b >>= 1
    return p


def aes_sbox():
    s = []
    for x in range(256):
        inv = 0
        if x:
            inv = next(y for y in range(1, 256) if gmul(x, y) == 1)
        r = inv
        for k in range(1, 5):
            r ^= ((inv << k) | (inv >> (8 - k))) & 0xFF
        s.append(r ^ 0x63)
    return s


# ------------------------------------------------- tower field arithmetic on ints
# GF(4) = GF(2)[z]/(z^2+z+1): element (a1 a0) as 2-bit int a1*2 + a0.
def g4mul(a, b):
    return gmul(a, b, 0b111, 2)


# GF(16) = GF(4)[w]/(w^2 + w + mu): element A1*w + A0 as (A1 << 2) | A0.
def g16mul(a, b, mu):
    a1, a0, b1, b0 = a >> 2, a & 3, b >> 2, b & 3
    p, q, r = g4mul(a1, b1), g4mul(a0, b0), g4mul(a1 ^ a0, b1 ^ b0)
    return ((r ^ q) << 2) | (q ^ g4mul(mu, p))


# GF(256) = GF(16)[y]/(y^2 + y + lam): element C1*y + C0 as (C1 << 4) | C0.
def g256mul(a, b, mu, lam):
    a1, a0, b1, b0 = a >> 4, a & 15, b >> 4, b & 15
    p, q, r = g16mul(a1, b1, mu), g16mul(a0, b0, mu), g16mul(a1 ^ a0, b1 ^ b0, mu)
    return ((r ^ q) << 4) | (q ^ g16mul(lam, p, mu))


def g256pow(a, e, mu, lam):
    r = 1
    while e:
        if e & 1:
            r = g256mul(r, a, mu, lam)
        a = g256mul(a, a, mu, lam)
        e >>= 1
    return r


def irreducible_quadratic(c, mul, size):
    """y^2 + y + c has no root in the field of `size` elements."""
    return all(mul(y, y) ^ y ^ c for y in range(size))


# ------------------------------------------------------------------- GF(2) matrices
def mat_inv(cols):
    """cols[i] = image of basis vector i (8-bit ints); returns the inverse map's cols."""
    n = len(cols)
    rows = [sum(((cols[j] >> i) & 1) << j for j in range(n)) | (1 << (n + i)) for i in range(n)]
    for c in range(n):
        piv = next(r for r in range(c, n) if (rows[r] >> c) & 1)
        rows[c], rows[piv] = rows[piv], rows[c]
        for r in range(n):
            if r != c and (rows[r] >> c) & 1:
                rows[r] ^= rows[c]
    inv_rows = [rows[i] >> n for i in range(n)]
    return [sum(((inv_rows[i] >> j) & 1) << i for i in range(n)) for j in range(n)]


def apply_cols(cols, x):
    r = 0
    for j, c in enumerate(cols):
        if (x >> j) & 1:
            r ^= c
    return r


# ------------------------------------------------------------------------- circuits
class Circuit:
    """Wires carry 256-bit truth tables; linear values are sets of wire ids (XOR)."""

    def __init__(self):
        self.tt = [sum(((x >> i) & 1) << x for x in range(256)) for i in range(8)]
        self.gates = []  # (op, out, a, b)
        self.cache = {frozenset([i]): i for i in range(8)}
        self.base = {i: frozenset([i]) for i in range(8)}  # wire -> XOR of base wires

    def new(self, op, a, b):
        w = len(self.tt)
        self.tt.append(self.tt[a] ^ self.tt[b] if op == "^" else self.tt[a] & self.tt[b])
        self.gates.append((op, w, a, b))
        self.base[w] = self.base[a] ^ self.base[b] if op == "^" else frozenset([w])
        return w

    def materialize(self, lins):
        """Wire ids for a batch of linear values, sharing XORs (Paar's heuristic)."""
        todo = {}
        for s in lins:
            s = frozenset(s)
            if s not in self.cache and s:
                todo[s] = set(s)
        rows = list(todo.items())
        while True:
            cnt = {}
            for _, cur in rows:
                if len(cur) >= 2:
                    for a, b in itertools.combinations(sorted(cur), 2):
                        cnt[(a, b)] = cnt.get((a, b), 0) + 1
            if not cnt:
                break
            (a, b), _ = max(cnt.items(), key=lambda kv: (kv[1], -kv[0][0], -kv[0][1]))
            key = self.base[a] ^ self.base[b]
            w = self.cache.get(key)
            if w is None:
                w = self.new("^", a, b)
                self.cache[key] = w
            for _, cur in rows:
                if a in cur and b in cur:
                    cur.discard(a)
                    cur.discard(b)
                    cur.add(w)
        for s, cur in rows:
            self.cache[s] = next(iter(cur))
        return [self.cache[frozenset(s)] if s else None for s in lins]

    def AND(self, a, b):
        wa, wb = self.materialize([a, b])
        w = self.new("&", wa, wb)
        self.cache[frozenset([w])] = w
        return {w}


def lin_xor(*xs):
    r = set()
    for x in xs:
        r ^= x
    return r


# Linear values in tower coordinates: a GF(4) element is a pair (hi, lo) of linear
# values, a GF(16) element a pair of GF(4) elements, and so on.
def l4_add(a, b):
    return (lin_xor(a[0], b[0]), lin_xor(a[1], b[1]))


def l4_mulconst(c, a):
    """c * a in GF(4) for a constant c, linear in a's bits."""
    # the image of the basis: c*z (hi bit) and c*1 (lo bit)
    cz, c1 = g4mul(c, 2), g4mul(c, 1)
    hi = lin_xor(*([a[0]] if cz & 2 else []), *([a[1]] if c1 & 2 else []))
    lo = lin_xor(*([a[0]] if cz & 1 else []), *([a[1]] if c1 & 1 else []))
    return (hi, lo)


def l4_sq(a):
    return l4_mulconst_fn(lambda x: g4mul(x, x), a)


def l4_mulconst_fn(f, a):
    """Any GF(2)-linear map f on GF(4), applied to linear values."""
    fz, f1 = f(2), f(1)
    hi = lin_xor(*([a[0]] if fz & 2 else []), *([a[1]] if f1 & 2 else []))
    lo = lin_xor(*([a[0]] if fz & 1 else []), *([a[1]] if f1 & 1 else []))
    return (hi, lo)


def c4_mul(C, a, b):
    """GF(4) product, Karatsuba: 3 ANDs."""
    p = C.AND(a[0], b[0])
    q = C.AND(a[1], b[1])
    r = C.AND(lin_xor(a[0], a[1]), lin_xor(b[0], b[1]))
    return (lin_xor(r, q), lin_xor(q, p))


def l16_lin(f, A):
    """Any GF(2)-linear map f on GF(16) (as ints), applied to linear values."""
    bits = [A[0][0], A[0][1], A[1][0], A[1][1]]  # value bits 3,2,1,0
    imgs = [f(8), f(4), f(2), f(1)]
    out = []
    for ob in (3, 2, 1, 0):
        out.append(lin_xor(*[bits[i] for i in range(4) if (imgs[i] >> ob) & 1]))
    return ((out[0], out[1]), (out[2], out[3]))


def l16_add(A, B):
    return (l4_add(A[0], B[0]), l4_add(A[1], B[1]))


def operands16(A):
    """The 9 linear values a GF(16) Karatsuba product ANDs for operand A."""
    out = []
    for x in (A[0], A[1], l4_add(A[0], A[1])):
        out += [x[0], x[1], lin_xor(x[0], x[1])]
    return out


def c16_mul(C, A, B, mu):
    C.materialize(operands16(A) + operands16(B))  # one batch: shared XORs
    P = c4_mul(C, A[0], B[0])
    Q = c4_mul(C, A[1], B[1])
    R = c4_mul(C, l4_add(A[0], A[1]), l4_add(B[0], B[1]))
    return (l4_add(R, Q), l4_add(Q, l4_mulconst(mu, P)))


def c16_inv(C, A, mu):
    """(A1 w + A0)^-1 = (A1 w + A0 + A1) * E^-1, E = mu A1^2 + A1 A0 + A0^2 in GF(4)."""
    A1, A0 = A
    sq = lambda x: g4mul(x, x)
    E = l4_add(l4_add(l4_mulconst_fn(lambda x: g4mul(mu, sq(x)), A1), c4_mul(C, A1, A0)),
               l4_mulconst_fn(sq, A0))
    Ei = l4_mulconst_fn(sq, E)  # inverse in GF(4) is the square (0 -> 0)
    return (c4_mul(C, A1, Ei), c4_mul(C, l4_add(A0, A1), Ei))


def build(mu, lam, beta):
    """S-box circuit (without the 0x63) for one tower choice; None if beta is no root."""
    # phi: AES basis x^i -> beta^i in the tower representation
    M = [g256pow(beta, i, mu, lam) for i in range(8)]
    if len(set(apply_cols(M, x) for x in range(256))) != 256:
        return None
    Minv = mat_inv(M)
    # affine matrix of FIPS-197 (without the constant), as columns
    Acols = []
    for j in range(8):
        b = 1 << j
        r = b
        for k in range(1, 5):
            r ^= ((b << k) | (b >> (8 - k))) & 0xFF
        Acols.append(r)
    N = [apply_cols(Acols, apply_cols(Minv, 1 << j)) for j in range(8)]  # A * M^-1
    C = Circuit()
    # tower coordinates of the input: bit t of phi(x) = XOR of x_i with (M[i] >> t) & 1
    v = [set(i for i in range(8) if (M[i] >> t) & 1) for t in range(8)]
    A1 = ((v[7], v[6]), (v[5], v[4]))
    A0 = ((v[3], v[2]), (v[1], v[0]))
    sq16 = lambda x: g16mul(x, x, mu)
    # the top linear layer: every AND operand that is linear in the input, in one batch
    C.materialize(operands16(A1) + operands16(A0) + operands16(l16_add(A0, A1)))
    # Delta = lam A1^2 + A1 A0 + A0^2 in GF(16)
    D = l16_add(l16_add(l16_lin(lambda x: g16mul(lam, sq16(x), mu), A1), c16_mul(C, A1, A0, mu)),
                l16_lin(sq16, A0))
    Di = c16_inv(C, D, mu)
    C1 = c16_mul(C, A1, Di, mu)
    C0 = c16_mul(C, l16_add(A0, A1), Di, mu)
    tower_bits = [C0[1][1], C0[1][0], C0[0][1], C0[0][0], C1[1][1], C1[1][0], C1[0][1], C1[0][0]]
    outs = [lin_xor(*[tower_bits[t] for t in range(8) if (N[t] >> j) & 1]) for j in range(8)]
    wires = C.materialize(outs)
    return C, wires



# ------------------------------------------------------------ 3-input LUT mapping
# gfx950's v_bitop3_b32 evaluates any boolean function of three 32-bit operands in one
# instruction (the 8-bit truth table is an immediate).  Covering the AND/XOR circuit
# with 3-input cuts (area flow, then exact-area recovery, as FPGA LUT mappers do) turns
# it into the fewest such instructions.
def lut_map(gates, outputs, K=3):
    op = {w: (o, a, b) for o, w, a, b in gates}
    order = [w for _, w, _, _ in gates]
    is_pi = lambda w: w not in op
    cuts = {}

    def cuts_of(w):
        if w in cuts:
            return cuts[w]
        if is_pi(w):
            cuts[w] = [frozenset([w])]
            return cuts[w]
        _, a, b = op[w]
        cs = set()
        for c1 in cuts_of(a):
            for c2 in cuts_of(b):
                u = c1 | c2
                if len(u) <= K:
                    cs.add(u)
        cs = [c for c in cs if not any(o < c for o in cs)]  # drop dominated cuts
        cuts[w] = cs + [frozenset([w])]
        return cuts[w]

    for w in order:
        cuts_of(w)
    fanout = {w: 0 for w in list(op) + list(range(8))}
    for w in order:
        _, a, b = op[w]
        fanout[a] += 1
        fanout[b] += 1
    for w in outputs:
        fanout[w] += 1
    af, best = {}, {}
    for w in range(8):
        af[w] = 0.0
    for w in order:
        opts = [c for c in cuts[w] if c != frozenset([w])]
        scored = [(1 + sum(af[l] / max(1, fanout[l]) for l in c), len(c), sorted(c), c) for c in opts]
        scored.sort(key=lambda t: (t[0], t[1], t[2]))
        af[w], best[w] = scored[0][0], scored[0][3]
    ref = {w: 0 for w in fanout}

    def do_ref(w):
        a = 1
        for l in best[w]:
            if not is_pi(l):
                if ref[l] == 0:
                    a += do_ref(l)
            ref[l] += 1
        return a

    def do_deref(w):
        a = 1
        for l in best[w]:
            ref[l] -= 1
            if not is_pi(l) and ref[l] == 0:
                a += do_deref(l)
        return a

    for w in outputs:
        if not is_pi(w):
            if ref[w] == 0:
                do_ref(w)
        ref[w] += 1
    for _ in range(3):  # exact-area recovery
        for w in order:
            if ref[w] == 0:
                continue
            do_deref(w)
            cand = []
            for c in cuts[w]:
                if c == frozenset([w]):
                    continue
                best[w] = c
                a = do_ref(w)
                do_deref(w)
                cand.append((a, len(c), sorted(c), c))
            cand.sort(key=lambda t: (t[0], t[1], t[2]))
            best[w] = cand[0][3]
            do_ref(w)
    mapped = [w for w in order if ref[w] > 0]

    def tt(w, leaves):
        """Truth table of w over its cut leaves (leaf 0 the most significant variable)."""
        pat = {l: p for l, p in zip(leaves, (0xF0, 0xCC, 0xAA))}
        memo = {}

        def ev(x):
            if x in pat:
                return pat[x]
            if x in memo:
                return memo[x]
            o, a, b = op[x]
            v = ev(a) ^ ev(b) if o == "^" else ev(a) & ev(b)
            memo[x] = v
            return v

        return ev(w) & 0xFF

    luts = []
    for w in mapped:
        leaves = sorted(best[w])
        luts.append((w, leaves, tt(w, leaves)))
    return luts


def check_luts(luts, outputs, S):
    val = {i: sum(((x >> i) & 1) << x for x in range(256)) for i in range(8)}
    full = (1 << 256) - 1
    for w, leaves, imm in luts:
        ops = [val[l] for l in leaves] + [val[leaves[0]]] * (3 - len(leaves))
        r = 0
        for m in range(8):
            if (imm >> m) & 1:
                t = full
                for k, v in enumerate(ops):
                    t &= v if (m >> (2 - k)) & 1 else full ^ v
                r |= t
        val[w] = r
    for j in range(8):
        want = sum((((S[x] ^ 0x63) >> j) & 1) << x for x in range(256))
        assert val[outputs[j]] == want, f"LUT output bit {j} wrong"


def main():
    S = aes_sbox()
    best = None
    for mu in range(1, 4):
        if not irreducible_quadratic(mu, g4mul, 4):
            continue
        for lam in range(1, 16):
            if not irreducible_quadratic(lam, lambda a, b: g16mul(a, b, mu), 16):
                continue
            for beta in range(2, 256):
                # beta must satisfy the AES polynomial x^8 + x^4 + x^3 + x + 1
                pw = [g256pow(beta, e, mu, lam) for e in (8, 4, 3, 1)]
                if pw[0] ^ pw[1] ^ pw[2] ^ pw[3] ^ 1:
                    continue
                r = build(mu, lam, beta)
                if r is None:
                    continue
                C, wires = r
                nx = sum(1 for g in C.gates if g[0] == "^")
                na = sum(1 for g in C.gates if g[0] == "&")
                luts = lut_map(C.gates, wires)
                if best is None or (len(luts), nx + na) < best[0]:
                    best = ((len(luts), nx + na), nx, na, mu, lam, beta, C, wires, luts)
    _, nx, na, mu, lam, beta, C, wires, luts = best
    check_luts(luts, wires, S)
    # exhaustive check on all 256 inputs
    for j in range(8):
        want = sum((((S[x] ^ 0x63) >> j) & 1) << x for x in range(256))
        assert C.tt[wires[j]] == want, f"output bit {j} wrong"
    # keep only gates the outputs need
    need = set(wires)
    for op, w, a, b in reversed(C.gates):
        if w in need:
            need.update((a, b))
    gates = [g for g in C.gates if g[1] in need]
    lines = [
        "// aes_sbox_bs.h — GENERATED by scripts/gen_aes_sbox.py; do not edit.",
        "//",
        "// Bitsliced AES S-box without its affine constant 0x63 (folded into the round",
        "// keys by k_aes.hip): x[i] holds bit i of the input byte of every slice; on",
        f"// return x[i] holds bit i of S(x) ^ 0x63.  Tower GF(((2^2)^2)^2) with mu = {mu},",
        f"// lambda = {lam}, beta = {beta} (see the script): {sum(g[0] == '^' for g in gates)} XOR + "
        f"{sum(g[0] == '&' for g in gates)} AND, covered by",
        f"// {len(luts)} three-input functions (one v_bitop3_b32 each on gfx950); circuit and",
        "// cover checked on all 256 inputs when generated.  No table, no branch: constant time.",
        "#pragma once",
        "#include <hip/hip_runtime.h>",
        "#include <stdint.h>",
        "",
        "// f(a, b, c) bitwise, truth table T indexed by (a << 2) | (b << 1) | c",
        "template <unsigned T>",
        "__host__ __device__ __forceinline__ uint32_t lut3(uint32_t a, uint32_t b, uint32_t c) {",
        "#if __HIP_DEVICE_COMPILE__",
        "    return __builtin_amdgcn_bitop3_b32(a, b, c, T);",
        "#else",
        "    uint32_t r = 0;",
        "    for (unsigned m = 0; m < 8; ++m)",
        "        if ((T >> m) & 1u)",
        "            r |= ((m & 4) ? a : ~a) & ((m & 2) ? b : ~b) & ((m & 1) ? c : ~c);",
        "    return r;",
        "#endif",
        "}",
        "",
        "__host__ __device__ __forceinline__ void aes_sbox_bs(uint32_t x[8]) {",
    ]
    for i in range(8):
        lines.append(f"    const uint32_t w{i} = x[{i}];")
    for w, leaves, imm in luts:
        ops = [f"w{l}" for l in leaves] + [f"w{leaves[0]}"] * (3 - len(leaves))
        lines.append(f"    const uint32_t w{w} = lut3<0x{imm:02x}>({', '.join(ops)});")
    for j in range(8):
        lines.append(f"    x[{j}] = w{wires[j]};")
    lines.append("}")
    # the same circuit as two-input gates, for the host key schedule (no bitop3 there)
    lines += ["", "// Host form: the AND/XOR circuit itself.",
              "inline void aes_sbox_gates(uint32_t x[8]) {"]
    for i in range(8):
        lines.append(f"    const uint32_t w{i} = x[{i}];")
    for op, w, a, b in gates:
        lines.append(f"    const uint32_t w{w} = w{a} {op} w{b};")
    for j in range(8):
        lines.append(f"    x[{j}] = w{wires[j]};")
    lines.append("}")
    with open(OUT, "w") as f:
        f.write("\n".join(lines) + "\n")
    print(f"mu={mu} lambda={lam} beta={beta}: {nx} XOR + {na} AND, {len(luts)} LUT3 -> {OUT}",
          file=sys.stderr)


if __name__ == "__main__":
    main()
