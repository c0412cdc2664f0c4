"""Dynamic VALU instructions per wave per set of the half-split c2 kernel's generated
blocks (bs8_small.inc; diagnostic): per-wave variants averaged, transposes, exchange
writes excluded.  usage: set_valu.py [bs8_small.inc]"""
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "rsmt2d_amd/csrc/bs8_small.inc"
text = open(path).read()


def body(name):
    return re.search(r"void %s\(.*?\{(.*?)\n\}" % name, text, re.S).group(1)


def valu(t):
    return len(re.findall(r'"v_', t))


def per_wave(name):
    b = body(name)
    parts = re.split(r"\.L%s\d_%%=:" % name, b)
    return sum(valu(p) for p in parts[1:]) / 8.0


blocks = {
    "small ifft h0": per_wave("small_ifft_h0_all"), "small ifft h1": per_wave("small_ifft_h1_all"),
    "small fft h0": per_wave("small_fft_h0_all"), "small fft h1": per_wave("small_fft_h1_all"),
    "large ifft h0 (ph_w1_lifft0)": valu(body("ph_w1_lifft0")), "lmid": valu(body("lmid_all")),
    "large fft h1 (ph_w0_lfft1)": valu(body("ph_w0_lfft1")),
    "transposes (tp_fwd x8, ph_w0_tr1, ph_w1_tr0, tp_inv x8)": 8 * valu(body("tp_fwd_dev")) + valu(body("ph_w0_tr1"))
    + valu(body("ph_w1_tr0")) + 8 * valu(body("tp_inv_dev")),
}
for k, v in blocks.items():
    print(f"{k:58s} {v:8.1f}")
print(f"{'total':58s} {sum(blocks.values()):8.1f}")
