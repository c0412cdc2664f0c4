"""CPU check of the GENERATED device butterflies the bit-sliced M = 128 encode
kernel executes (rsmt2d_amd/csrc/bs8_asm.inc and bs8_small.inc, written by
gen/gen_bs8_asm.cpp and gen/gen_bs8_small.cpp).  Every v_xor_b32 / v_bitop3_b32
line is parsed and executed on random bit-planes and the result compared with the
butterfly computed byte by byte from the oracle's GF(2^8) tables (klauspost
leopard8 restatement, SURVEY.md A.4: IFFT_DIT2 y ^= x; x ^= y*exp(L) --
FFT_DIT2 x ^= y*exp(L); y ^= x -- L == 255 XOR only).  The GPU code never runs
here: this pins the instruction text the kernel runs, shared-temporary networks
and the merged middle butterfly included."""
import os
import re

import numpy as np
import pytest

import oracle

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rsmt2d_amd", "csrc")
INS = re.compile(r'"(v_xor_b32|v_bitop3_b32) %(\d+), %(\d+), %(\d+)(?:, %(\d+) bitop3:0x96)?')


def parse(text):
    ops = []
    for m in INS.finditer(text):
        c = int(m.group(5)) if m.group(5) else -1
        assert (m.group(1) == "v_bitop3_b32") == (c >= 0), m.group(0)
        ops.append((int(m.group(2)), int(m.group(3)), int(m.group(4)), c))
    return ops


def execute(ops, regs):
    for d, a, b, c in ops:
        regs[d] = regs[a] ^ regs[b] ^ (regs[c] if c >= 0 else 0)


@pytest.fixture(scope="module")
def gf():
    exp, log, skew, _ = oracle.tables8()
    exp, log = exp.astype(np.int64), log.astype(np.int64)

    def mul(v, L):  # v * exp(L), Leopard mulLog; L == 255 is the zero multiplier
        if L == 255:
            return np.zeros_like(v)
        s = log[v] + L
        s = (s + (s >> 8)) & 255
        return np.where(v == 0, 0, exp[s]).astype(np.uint8)
    return mul, [int(x) for x in skew]


def planes(b):  # 32 bytes -> 8 u32 planes (bit n of plane i = bit i of byte n)
    bits = np.unpackbits(b[:, None], axis=1, bitorder="little")
    return [int(np.packbits(bits[:, i], bitorder="little").view("<u4")[0]) for i in range(8)]


def unplanes(p):
    return np.array([sum(((p[i] >> n) & 1) << i for i in range(8)) for n in range(32)], np.uint8)


def butterfly(kind, L, x, y, mul):
    if kind == "ifft2_asm":
        y = y ^ x
        x = x ^ mul(y, L)
    elif kind == "fft2_asm":
        x = x ^ mul(y, L)
        y = y ^ x
    else:  # mid2_asm
        y = y ^ x
        x = x ^ mul(y, L)
        y = y ^ x
    return x, y


@pytest.mark.parametrize("name", ["ifft2_asm", "fft2_asm", "mid2_asm"])
def test_butterfly_blocks(gf, name):
    mul, _ = gf
    text = open(os.path.join(CSRC, "bs8_asm.inc")).read()
    blocks = re.findall(r"void %s<(\d+)>\(.*?\{(.*?)\n\}" % name, text, re.S)
    assert sorted(int(L) for L, _ in blocks) == list(range(256))
    rng = np.random.default_rng(8)
    for L, body in blocks:
        L = int(L)
        x = rng.integers(0, 256, 32, dtype=np.uint8)
        y = rng.integers(0, 256, 32, dtype=np.uint8)
        regs = planes(x) + planes(y) + [int(v) for v in rng.integers(0, 2**32, 8)]  # garbage temporaries
        execute(parse(body), regs)
        wx, wy = butterfly(name, L, x, y, mul)
        assert unplanes(regs[:8]).tobytes() == wx.tobytes(), (name, L)
        assert unplanes(regs[8:16]).tobytes() == wy.tobytes(), (name, L)


@pytest.mark.parametrize("name,inverse", [("small_ifft_all", True), ("small_fft_all", False)])
def test_small_layer_blocks(gf, name, inverse):
    """The per-wave small layers (symbols e = 16A + j, d = 1, 2, 4; bs8.hpp)."""
    mul, skew = gf
    text = open(os.path.join(CSRC, "bs8_small.inc")).read()
    fn = re.search(r"void %s\(.*?\{(.*?)\n\}" % name, text, re.S).group(1)
    parts = re.split(r"\.L%s(\d)_%%=:" % name, fn)
    bodies = {int(parts[i]): parts[i + 1] for i in range(1, len(parts), 2)}
    assert sorted(bodies) == list(range(8))
    rng = np.random.default_rng(9)
    for A, body in bodies.items():
        sym = [rng.integers(0, 256, 32, dtype=np.uint8) for _ in range(16)]
        regs = sum((planes(s) for s in sym), []) + [int(v) for v in rng.integers(0, 2**32, 8)]
        execute(parse(body), regs)
        ref = [s.copy() for s in sym]
        for d in ((1, 2, 4) if inverse else (4, 2, 1)):
            for b in range(0, 16, 2 * d):
                L = skew[127 + 16 * A + b + d] if inverse else skew[-1 + 16 * A + b + d]
                for q in range(d):
                    ref[b + q], ref[b + q + d] = butterfly("ifft2_asm" if inverse else "fft2_asm", L,
                                                           ref[b + q], ref[b + q + d], mul)
        for j in range(16):
            assert unplanes(regs[8 * j:8 * j + 8]).tobytes() == ref[j].tobytes(), (name, A, j)


@pytest.mark.parametrize("G", [0, 1])
@pytest.mark.parametrize("name,inverse", [("small_ifft_h%d_all", True), ("small_fft_h%d_all", False)])
def test_half_split_small_layer_blocks(gf, name, inverse, G):
    """The half-split schedule's small layers (layout S': register b of half G of
    wave A holds e = b + 8A + 64G; d = 1, 2, 4 on b; bs8.hpp small_ifft_h)."""
    mul, skew = gf
    name = name % G
    text = open(os.path.join(CSRC, "bs8_small.inc")).read()
    fn = re.search(r"void %s\(.*?\{(.*?)\n\}" % name, text, re.S).group(1)
    parts = re.split(r"\.L%s(\d)_%%=:" % name, fn)
    bodies = {int(parts[i]): parts[i + 1] for i in range(1, len(parts), 2)}
    assert sorted(bodies) == list(range(8))
    rng = np.random.default_rng(10 + G)
    for A, body in bodies.items():
        sym = [rng.integers(0, 256, 32, dtype=np.uint8) for _ in range(8)]
        regs = sum((planes(s) for s in sym), []) + [int(v) for v in rng.integers(0, 2**32, 8)]
        execute(parse(body), regs)
        ref = [s.copy() for s in sym]
        for d in ((1, 2, 4) if inverse else (4, 2, 1)):
            for b in range(0, 8, 2 * d):
                e0 = 8 * A + 64 * G + b + d
                L = skew[127 + e0] if inverse else skew[-1 + e0]
                for q in range(d):
                    ref[b + q], ref[b + q + d] = butterfly("ifft2_asm" if inverse else "fft2_asm", L,
                                                           ref[b + q], ref[b + q + d], mul)
        for j in range(8):
            assert unplanes(regs[8 * j:8 * j + 8]).tobytes() == ref[j].tobytes(), (name, A, j)


# --- bytes <-> planes transposes of the half-split kernel (gen_bs8_small.cpp tp_ops) ---
GEN = re.compile(r'"(v_alignbit_b32|v_bitop3_b32|v_xor_b32) %(\d+), %(\d+), %(\d+)(?:, (?:%(\d+)|(\d+)))?'
                 r'(?: bitop3:(0x[0-9a-f]+))?')
M32 = 0xFFFFFFFF


def run_valu(text, regs):
    """Execute the VALU text of a generated block (v_alignbit_b32, v_bitop3_b32 XOR3 /
    select, v_xor_b32) on a register dict; LDS instructions are skipped."""
    n = 0
    for m in GEN.finditer(text):
        op, d, a, b = m.group(1), int(m.group(2)), int(m.group(3)), int(m.group(4))
        if op == "v_alignbit_b32":
            regs[d] = (((regs[a] << 32) | regs[b]) >> int(m.group(6))) & M32
        elif op == "v_xor_b32":
            regs[d] = regs[a] ^ regs[b]
        else:
            c = regs[int(m.group(5))]
            if m.group(7) == "0x96":
                regs[d] = regs[a] ^ regs[b] ^ c
            else:
                assert m.group(7) == "0xd8", m.group(0)
                regs[d] = (regs[b] & c) | (regs[a] & ~c & M32)  # S2 ? S1 : S0
        n += 1
    return n


def layout_of(fwd_words):
    """Bit position of byte (r, b) in the planes, from single-byte probes; None if the
    planes do not share one layout."""
    pos = {}
    for r in range(8):
        for b in range(4):
            w = [0] * 8
            w[r] = 0xFF << (8 * b)
            out = fwd_words(w)
            bits = {o.bit_length() - 1 for o in out}
            if any(bin(o).count("1") != 1 for o in out) or len(bits) != 1:
                return None
            pos[(r, b)] = bits.pop()
    return pos


@pytest.fixture(scope="module")
def small_text():
    return open(os.path.join(CSRC, "bs8_small.inc")).read()


def block(text, name):
    return re.search(r"void %s\(.*?\{(.*?)\n\}" % name, text, re.S).group(1)


def tp_fn(text, name):
    body = block(text, name)
    masks = {10: 0xF0F0F0F0, 11: 0xCCCCCCCC, 12: 0xAAAAAAAA}

    def f(w):
        regs = dict(enumerate(w))
        regs.update({8: 0xDEADBEEF, 9: 0x12345678})
        regs.update(masks)
        run_valu(body, regs)
        return [regs[i] for i in range(8)]
    return f, body


def test_transposes_share_one_layout_and_invert(small_text):
    fwd, fb = tp_fn(small_text, "tp_fwd_dev")
    inv, ib = tp_fn(small_text, "tp_inv_dev")
    # 12 rotations + 5 fix-ups + 24 selects each way
    assert fb.count("v_alignbit_b32") == 17 and fb.count("bitop3:0xd8") == 24
    assert ib.count("v_alignbit_b32") == 17 and ib.count("bitop3:0xd8") == 24
    pos = layout_of(fwd)
    assert pos is not None and sorted(pos.values()) == list(range(32))
    rng = np.random.default_rng(11)
    for _ in range(64):
        w = [int(x) for x in rng.integers(0, 2**32, 8, dtype=np.uint64)]
        planes_ = fwd(w)
        for (r, b), x in pos.items():
            byte = (w[r] >> (8 * b)) & 0xFF
            for p in range(8):
                assert (planes_[p] >> x) & 1 == (byte >> p) & 1
        assert inv(planes_) == w


def phase_operands(body):
    """Temporaries (garbage) and the six SGPR masks of a generated phase block (the
    masks follow the block's temporaries, gen_bs8_small.cpp emit_phase)."""
    nt = len(re.findall(r'"=&v"\(t\d+\)', body))
    regs = {128 + t: 0x9E3779B9 * (t + 1) & M32 for t in range(nt)}
    masks = [int(m, 16) for m in re.findall(r'"s"\((0x[0-9A-Fa-f]+)u\)', body)]  # in operand order
    for i, m in enumerate(masks):
        regs[128 + nt + i] = m
    return regs


@pytest.mark.parametrize("name,V,kind", [("ph_w1_lifft0", 0, "ifft2_asm"), ("ph_w0_lfft1", 1, "fft2_asm")])
def test_phase_large_layers(gf, small_text, name, V, kind):
    """The large IFFT / FFT layers of one half (layout L: register h of wave g holds
    e = g + 8h; d = 8h-strides 1, 2, 4 within the half, bs8.hpp large_ifft_h/large_fft_h),
    interleaved with the other half's exchange writes."""
    mul, skew = gf
    body = block(small_text, name)
    rng = np.random.default_rng(13 + V)
    sym = [rng.integers(0, 256, 32, dtype=np.uint8) for _ in range(16)]
    regs = dict(enumerate(sum((planes(x) for x in sym), [])))
    regs.update(phase_operands(body))
    run_valu(body, regs)
    ref = [x.copy() for x in sym]
    for dh in ((1, 2, 4) if kind == "ifft2_asm" else (4, 2, 1)):
        for bb in range(0, 8, 2 * dh):
            hb = 8 * V + bb
            L = skew[127 + 8 * hb + 8 * dh] if kind == "ifft2_asm" else skew[-1 + 8 * hb + 8 * dh]
            for q in range(dh):
                ref[hb + q], ref[hb + q + dh] = butterfly(kind, L, ref[hb + q], ref[hb + q + dh], mul)
    for j in range(16):
        assert unplanes([regs[8 * j + i] for i in range(8)]).tobytes() == ref[j].tobytes(), (name, j)


@pytest.mark.parametrize("name,V,inverse", [("ph_w0_tr1", 1, False), ("ph_w1_tr0", 0, True)])
def test_phase_transposes(small_text, name, V, inverse):
    """The transposes interleaved with the exchange writes of the other half."""
    body = block(small_text, name)
    fwd, _ = tp_fn(small_text, "tp_fwd_dev")
    inv, _ = tp_fn(small_text, "tp_inv_dev")
    rng = np.random.default_rng(12)
    X = [int(x) for x in rng.integers(0, 2**32, 128, dtype=np.uint64)]
    regs = dict(enumerate(X))
    regs.update(phase_operands(body))
    assert run_valu(body, regs) == 8 * 41
    for j in range(16):
        got = [regs[8 * j + i] for i in range(8)]
        want = X[8 * j:8 * j + 8]
        if j // 8 == V:
            want = (inv if inverse else fwd)(want)
        assert got == want, (name, j)


def test_lmid_block(gf, small_text):
    """Large IFFT of half 1, the merged middle pair, large FFT of half 0 (bs8.hpp
    large_ifft_h<1> + large_mid + large_fft_h<0>) as one optimized block."""
    mul, skew = gf
    body = block(small_text, "lmid_all")
    rng = np.random.default_rng(14)
    sym = [rng.integers(0, 256, 32, dtype=np.uint8) for _ in range(16)]
    regs = dict(enumerate(sum((planes(x) for x in sym), [])))
    regs.update({128 + t: (0x9E3779B9 * (t + 1)) & M32 for t in range(8)})
    run_valu(body, regs)
    ref = [x.copy() for x in sym]
    for dh in (1, 2, 4):
        for bb in range(0, 8, 2 * dh):
            hb = 8 + bb
            for q in range(dh):
                ref[hb + q], ref[hb + q + dh] = butterfly("ifft2_asm", skew[127 + 8 * hb + 8 * dh], ref[hb + q],
                                                          ref[hb + q + dh], mul)
    exp, log, _, _ = oracle.tables8()
    e = lambda L: 0 if L == 255 else int(exp[L])
    s = e(skew[127 + 64]) ^ e(skew[63])
    mid = 255 if s == 0 else int(log[s])
    for q in range(8):
        ref[q], ref[q + 8] = butterfly("mid2_asm", mid, ref[q], ref[q + 8], mul)
    for dh in (4, 2, 1):
        for bb in range(0, 8, 2 * dh):
            for q in range(dh):
                ref[bb + q], ref[bb + q + dh] = butterfly("fft2_asm", skew[-1 + 8 * bb + 8 * dh], ref[bb + q],
                                                          ref[bb + q + dh], mul)
    for j in range(16):
        assert unplanes([regs[8 * j + i] for i in range(8)]).tobytes() == ref[j].tobytes(), j
