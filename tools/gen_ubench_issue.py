# generate tools/ubench_issue.hip: instruction-sequence issue-cost probes with in-kernel clock
A = "v_alignbit_b32 v{d}, v{d}, v{d}, 16"
X = "v_xor_b32 v{d}, v{d}, v73"
XE = "v_xor_b32_e64 v{d}, v{d}, v73"
B3 = "v_bitop3_b32 v{d}, v{d}, v73, 0 bitop3:0x96"
D3 = "v_add3_u32 v{d}, v{d}, v73, v78"
AD = "v_add_u32 v{d}, v{d}, v73"
ADE = "v_add_u32_e64 v{d}, v{d}, v73"
MV = "v_mov_b32 v{d}, v73"
LS = "v_lshrrev_b32 v{d}, 7, v{d}"
PM = "v_perm_b32 v{d}, v{d}, v{d}, v78"
FA = "v_add_f32 v{d}, v{d}, v73"
FM = "v_fma_f32 v{d}, v{d}, v73, v78"
PF = "v_pk_fma_f32 v[{d}:{d1}], v[{d}:{d1}], v[74:75], v[76:77]"
PA = "v_pk_add_f32 v[{d}:{d1}], v[{d}:{d1}], v[74:75]"
CM = "v_cndmask_b32 v{d}, v{d}, v73, vcc"
SN = "s_nop 0"
seqs = {
 "A*7 X": [A]*7 + [X], "A*6 X*2": [A]*6 + [X]*2, "A*2 X*6": [A]*2 + [X]*6, "A X*7": [A] + [X]*7,
 "A MV*7": [A] + [MV]*7, "X*4 MV*4": [X]*4 + [MV]*4, "A MV X MV": [A, MV, X, MV]*2,
 "FA": [FA]*8, "FM": [FM]*8, "PF": [PF]*8, "PA": [PA]*8, "A FA": [A, FA]*4, "A FM": [A, FM]*4,
 "A PF": [A, PF]*4, "A CM": [A, CM]*4, "A SN": [A, SN]*4, "X FA": [X, FA]*4,

 "X": [X]*8, "XE": [XE]*8, "B3": [B3]*8, "AD": [AD]*8, "A": [A]*8, "D3": [D3]*8, "PM": [PM]*8,
 "A X": [A, X]*4, "A XE": [A, XE]*4, "A B3": [A, B3]*4, "A AD": [A, AD]*4, "A ADE": [A, ADE]*4,
 "A A X X": [A, A, X, X]*2, "A A XE XE": [A, A, XE, XE]*2, "AAAA XXXX": [A]*4+[X]*4,
 "A X X": [A, X, X, A, X, X, A, X], "A XE XE": [A, XE, XE, A, XE, XE, A, XE],
 "A MV": [A, MV]*4, "A LS": [A, LS]*4, "D3 AD": [D3, AD]*4, "D3 X": [D3, X]*4, "D3 A": [D3, A]*4,
 "X AD": [X, AD]*4, "XE ADE": [XE, ADE]*4, "X XE": [X, XE]*4,
}
regs = [40, 44, 48, 52, 56, 60, 64, 68]
out = []
names = []
for i, (name, seq) in enumerate(seqs.items()):
    body = "\\n".join(ins.format(d=regs[j], d1=regs[j] + 1) for j, ins in enumerate(seq))
    out.append(f'KLOOP(k{i}, "{body}\\n")')
    names.append((name, f"k{i}"))
src = open("/root/repo/tools/ubench_issue.tmpl").read()
src = src.replace("@KERNELS@", "\n".join(out))
src = src.replace("@TABLE@", ", ".join(f'{{"{n}", {k}}}' for n, k in names))
open("/root/repo/tools/ubench_issue.hip", "w").write(src)
