# generate tools/ubench_f64.hip: can integer adds move to the FP64 pipe next to the
# half-rate v_alignbit/v_add3 stream?  A u32 add is exact as a v_add_f64 of denormal
# doubles (hi dword 0 / small carry, low dword = the u32): low dword of the sum = a + b
# mod 2^32.  Probes: issue cost (in-kernel clock) of BLAKE3-G-shaped sequences with the
# adds as v_add3/v_add (today) vs v_add_f64; plus a bit-exactness check of the trick.
A = "v_alignbit_b32 v{d}, v{d}, v{d}, 16"
X = "v_xor_b32 v{d}, v{d}, v90"
D3 = "v_add3_u32 v{d}, v{d}, v90, v91"
AD = "v_add_u32 v{d}, v{d}, v90"
DA = "v_add_f64 v[{d}:{d1}], v[{d}:{d1}], v[92:93]"
DF = "v_fma_f64 v[{d}:{d1}], v[{d}:{d1}], v[94:95], v[92:93]"
FA = "v_add_f32 v{d}, v{d}, v90"
PK = "v_pack_b32_f16 v{d}, v{d}, v{d} op_sel:[1,0,0]"  # = rotr16 if it moves bits unchanged
seqs = {
    "DA": [DA] * 12,
    "A": [A] * 12,
    "A DA": [A, DA] * 6,
    "X DA": [X, DA] * 6,
    "A X DA": [A, X, DA] * 4,
    "A FA": [A, FA] * 6,
    # one BLAKE3 G as compiled today: 2 add3 + 2 add + 4 xor + 4 alignbit
    "G int": [D3, X, A, AD, X, A, D3, X, A, AD, X, A],
    # G with the adds on the FP64 pipe: a+b+x = 2 v_add_f64, c+d = 1
    "G f64": [DA, DA, X, A, DA, X, A, DA, DA, X, A, DA, X, A],
    # G with only c+d on FP64
    "G half": [D3, X, A, DA, X, A, D3, X, A, DA, X, A],
    "PK": [PK] * 12,
    "A PK": [A, PK] * 6,
    "X PK": [X, PK] * 6,
    # G with its rotate-by-16 as v_pack_b32_f16 (op_sel: high half first)
    "G pk16": [D3, X, PK, AD, X, A, D3, X, A, AD, X, A],
}
NCH = 12
out, names = [], []
for i, (name, seq) in enumerate(seqs.items()):
    body = "\\n".join(ins.format(d=40 + 2 * (j % NCH), d1=41 + 2 * (j % NCH)) for j, ins in enumerate(seq))
    out.append(f'KLOOP(k{i}, "{body}\\n", {len(seq)})')
    names.append((name, f"k{i}", len(seq)))
src = open("tools/ubench_f64.tmpl").read()
src = src.replace("@KERNELS@", "\n".join(out))
src = src.replace("@TABLE@", ", ".join(f'{{"{n}", {k}, {L}}}' for n, k, L in names))
open("tools/ubench_f64.hip", "w").write(src)
