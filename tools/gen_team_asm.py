#!/usr/bin/env python3
"""Generate nmpc_nav_control_amd/csrc/team_asm_gen.hpp: whole-block fused-DPP kernels of the team Riccati step.

Each block is one inline-asm statement holding every broadcast-FMA of a dense sub-step of the classic (fp64)
Riccati factorisation (v_fmac_f64_dpp / v_fmac_f32_dpp with row_newbcast). One block costs one s_nop (the
VALU-write -> DPP-read hazard can only involve instructions before the block: inside it only accumulators are
written and no accumulator is a DPP source), and the terms are ordered so that consecutive FMAs hit different
accumulators. Measured on MI355X (scratch microbenchmark, one wave per SIMD): v_fmac_f64_dpp 5.6 cycles,
s_nop 1 8.4 cycles, so per-term nops would cost more than the FMAs.

Usage: python tools/gen_team_asm.py [out]   (rewrites the header; `make` in csrc does not run it;
tests/test_codegen.py::test_team_asm_header_is_generated checks the committed header against generate())
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "nmpc_nav_control_amd", "csrc", "team_asm_gen.hpp")
SHAPES = [(7, 2), (11, 4)]  # (NX, NU): diff2amr / tric3amr, omni4amr
# leading rows of [B A] the column-form M block broadcasts (team_common.hpp m_block): the NGV state-dependent rows
# and theta's row, the densest constant one (7 of 9 / 13 of 15 columns: broadcasting it costs 2 more FMAs than its
# uniform-operand form and saves 7 / 13 uniform fp64 registers)
VAR_ROWS = {(7, 2): (3,), (11, 4): (3,)}
M = " row_mask:0xf bank_mask:0xf"


# fp64 (the default factorisation) or fp32 (the split-sigma fp32 factorisation of the single-direction team kernel,
# DESIGN.md section 5): instruction, C type and function-name suffix
TYPES = {"f64": ("v_fmac_f64_dpp", "v_mov_b64_dpp", "double", ""),
         "f32": ("v_fmac_f32_dpp", "v_mov_b32_dpp", "float", "_f32")}


def pg_block(nx, nu, t="f64"):
    # classic Riccati: pg[i] += bcast_{nu+i}(Prow[nu+l]) * Gd[l] (column v of P_{k+1} [B A]); lane nu+i holds row i
    # of P_{k+1}; operands: acc 0..nx-1 (+v), Prow x-part nx.., Gd 2nx..
    fma, _, ct, sfx = TYPES[t]
    lines = ["s_nop 1"]
    for l in range(nx):
        for i in range(nx):
            lines.append(f"{fma} %{i}, %{nx + l}, %{2 * nx + l} row_newbcast:{nu + i}{M}")
    outs = ", ".join(f'"+v"(acc[{i}])' for i in range(nx))
    ins = ", ".join([f'"v"(prow[{nu + l}])' for l in range(nx)] + [f'"v"(gd[{l}])' for l in range(nx)])
    body = "\\n\\t".join(lines)
    return (f"__device__ __forceinline__ void pg_block{sfx}_{nx}_{nu}({ct} (&acc)[{nx}], const {ct} (&prow)[{nx + nu}],"
            f" const {ct} (&gd)[{nx}])\n{{\n    asm(\"{body}\"\n        : {outs}\n        : {ins});\n}}\n")


def mrow_pg_block(nx, nu):
    # classic Riccati: Mr[j] += bcast_j(pg[i]) * Gd[i] (row r of [B A]' P [B A]: lane r holds column r of [B A]),
    # then md0 = bcast_0(Mr[0]), the first pivot; operands: Mr 0..nv-1 (+v), md0 (=v), pg .., Gd ..
    nv = nx + nu
    lines = ["s_nop 1"]
    for i in range(nx):
        for j in range(nv):
            lines.append(f"v_fmac_f64_dpp %{j}, %{nv + 1 + i}, %{nv + 1 + nx + i} row_newbcast:{j}{M}")
    lines.append("s_nop 1")
    lines.append(f"v_mov_b64_dpp %{nv}, %0 row_newbcast:0{M}")
    outs = ", ".join([f'"+v"(acc[{j}])' for j in range(nv)] + ['"=&v"(md0)'])
    ins = ", ".join([f'"v"(pg[{i}])' for i in range(nx)] + [f'"v"(gd[{i}])' for i in range(nx)])
    body = "\\n\\t".join(lines)
    return (f"__device__ __forceinline__ void mrow_pg_block_{nx}_{nu}(double (&acc)[{nv}], double& md0,"
            f" const double (&pg)[{nx}], const double (&gd)[{nx}])\n{{\n    asm(\"{body}\"\n        : {outs}\n"
            f"        : {ins});\n}}\n")


def mcol_var_block(nx, nu, ngv, t="f64"):
    # classic Riccati, column form of M = D + [B A]' P [B A] on lane j: acc[r] += bcast_r(Gd[i]) * pg[i] over the
    # ngv state-dependent rows i of [B A] (lane r holds column r of [B A], lane j column j of P [B A]); the constant
    # rows are the caller's uniform-operand FMAs (team_common.hpp m_block). Then md0 = bcast_0(acc[0]), the first
    # pivot. M is symmetric, so lane j's column j is its row j. Operands: acc 0..nv-1 (+v), md0 (=v), Gd.., pg..
    # fp64 NU = 2 also broadcasts M[1][1] and M[0][1] (m11, m10): both input pivots then come from the 2 x 2 block at
    # once (the second as det / M00), so their rsq chains run side by side (sqp_rti_team.hip P1); the fp32 form takes
    # its pivots in turn (each may carry a bounded state's barrier weight, team_common.hpp chol_split_f32)
    fma, mov, ct, sfx = TYPES[t]
    nv = nx + nu
    npv = 3 if (nu == 2 and t == "f64") else 1
    lines = ["s_nop 1"]
    for i in range(ngv):
        for r in range(nv):
            lines.append(f"{fma} %{r}, %{nv + npv + i}, %{nv + npv + ngv + i} row_newbcast:{r}{M}")
    lines.append("s_nop 1")
    lines.append(f"{mov} %{nv}, %0 row_newbcast:0{M}")
    if npv == 3:
        lines.append(f"{mov} %{nv + 1}, %1 row_newbcast:1{M}")
        lines.append(f"{mov} %{nv + 2}, %0 row_newbcast:1{M}")
    outs = ", ".join([f'"+v"(acc[{r}])' for r in range(nv)] + ['"=&v"(md0)'] +
                     (['"=&v"(m11)', '"=&v"(m10)'] if npv == 3 else []))
    ins = ", ".join([f'"v"(gd[{i}])' for i in range(ngv)] + [f'"v"(pg[{i}])' for i in range(ngv)])
    body = "\\n\\t".join(lines)
    extra = f", {ct}& m11, {ct}& m10" if npv == 3 else ""
    return (f"__device__ __forceinline__ void mcol_var_block{sfx}_{nx}_{nu}_{ngv}({ct} (&acc)[{nv}], {ct}& md0{extra},"
            f" const {ct} (&pg)[{nx}], const {ct} (&gd)[{nx}])\n{{\n    asm(\"{body}\"\n        : {outs}\n"
            f"        : {ins});\n}}\n")


def chol_update(nx, nu, t="f64"):
    # column j done: Lr[jp] -= bcast_jp(lj) * lj for jp > j, then pivot of column j+1 = bcast_{j+1}(Lr[j+1])
    fma, mov, ct, sfx = TYPES[t]
    nv = nx + nu
    out = []
    for j in range(nv - 1 if t == "f64" else nu):  # fp32: the input columns only (the split-sigma factor's pivots)
        lines = ["s_nop 1"]
        k = 0
        ops = []
        for jp in range(j + 1, nv):
            lines.append(f"{fma} %{k}, -%{nv - j - 1 + 1}, %{nv - j - 1 + 1} row_newbcast:{jp}{M}")
            ops.append(f'"+v"(lr[{jp}])')
            k += 1
        n = nv - j - 1
        # the pivot broadcast reads lr[j+1], written by the first FMA: two more VALU ops must separate them
        if n < 3:
            lines.append("s_nop 1")
        lines.append(f"{mov} %{n}, %0 row_newbcast:{j + 1}{M}")
        outs = ", ".join(ops + ['"=&v"(piv)'])
        body = "\\n\\t".join(lines)
        out.append(f"__device__ __forceinline__ void chol_update{sfx}_{nx}_{nu}_{j}({ct} (&lr)[{nv}], {ct} lj, {ct}& piv)\n"
                   f"{{\n    asm(\"{body}\"\n        : {outs}\n        : \"v\"(lj));\n}}\n")
    if t == "f32":
        cases = "\n".join(f"    if constexpr (J == {j}) chol_update_f32_{nx}_{nu}_{j}(lr, lj, piv);" for j in range(nu))
        out.append(f"template <int J>\n__device__ __forceinline__ void chol_update_f32_{nx}_{nu}(float (&lr)[{nv}], float lj,"
                   f" float& piv)\n{{\n{cases}\n}}\n")
        return "\n".join(out)
    # the same updates without the next pivot's broadcast (input columns j < nu, when the pivots are known up front)
    for j in range(nu):
        lines = ["s_nop 1"]
        ops = []
        for k, jp in enumerate(range(j + 1, nv)):
            lines.append(f"v_fmac_f64_dpp %{k}, -%{nv - j - 1}, %{nv - j - 1} row_newbcast:{jp}{M}")
            ops.append(f'"+v"(lr[{jp}])')
        body = "\\n\\t".join(lines)
        out.append(f"__device__ __forceinline__ void chol_update_np_{nx}_{nu}_{j}(double (&lr)[{nv}], double lj)\n"
                   f"{{\n    asm(\"{body}\"\n        : {', '.join(ops)}\n        : \"v\"(lj));\n}}\n")
    # dispatcher
    cases = "\n".join(f"    if constexpr (J == {j}) chol_update_{nx}_{nu}_{j}(lr, lj, piv);" for j in range(nv - 1))
    out.append(f"template <int J>\n__device__ __forceinline__ void chol_update_{nx}_{nu}(double (&lr)[{nv}], double lj,"
               f" double& piv)\n{{\n{cases}\n}}\n")
    return "\n".join(out)


def dot_f32(n, j0, name):
    # acc + sum_t bcast_{j0+t}(a) * b[t] as two interleaved partial sums (operands: p0, p1, a, b...)
    lines = ["s_nop 1"]
    for t in range(n):
        lines.append(f"v_fmac_f32_dpp %{t % 2}, %2, %{3 + t} row_newbcast:{j0 + t}{M}")
    ins = ", ".join(['"v"(a)'] + [f'"v"(b[{t}])' for t in range(n)])
    body = "\\n\\t".join(lines)
    return (f"__device__ __forceinline__ float {name}(float acc, float a, const float (&b)[{n}])\n{{\n"
            f"    float p1 = 0.0f;\n    asm(\"{body}\"\n        : \"+v\"(acc), \"+v\"(p1)\n        : {ins});\n"
            f"    return acc + p1;\n}}\n")


# ---- segmented Riccati master (sqp_rti_rowpar.hip SEG): n x n blocks on the state lanes off .. off + n - 1 of
# one 16-lane row, lane off + r holding row r of every matrix and element r of every vector

def mst_rowmul(n, off):
    # acc[c] (+|-)= bcast_{off+l}(B[c]) * a[l]: row r of A B (lane off+l holds row l of B); operands acc, B, a
    out = []
    for sign, nm in (("", "mst_rowmul"), ("-", "mst_rowmul_neg")):
        lines = ["s_nop 1"]
        for l in range(n):
            for c in range(n):
                lines.append(f"v_fmac_f64_dpp %{c}, {sign}%{n + c}, %{2 * n + l} row_newbcast:{off + l}{M}")
        outs = ", ".join(f'"+v"(acc[{c}])' for c in range(n))
        ins = ", ".join([f'"v"(b[{c}])' for c in range(n)] + [f'"v"(a[{l}])' for l in range(n)])
        body = "\\n\\t".join(lines)
        out.append(f"__device__ __forceinline__ void {nm}_{n}_{off}(double (&acc)[{n}], const double (&a)[{n}],"
                   f" const double (&b)[{n}])\n{{\n    asm(\"{body}\"\n        : {outs}\n        : {ins});\n}}\n")
    return "\n".join(out)


def mst_rowmul_lt(n, off):
    # acc[c] += bcast_{off+l}(b[c]) * a[l] for l >= c only: row r of A B with B lower triangular (b[c] = 0 on lane
    # off + l for c > l), or the lower triangle of A B where row r of A vanishes left of r (the master's L' V)
    lines = ["s_nop 1"]
    for l in range(n):
        for c in range(l + 1):
            lines.append(f"v_fmac_f64_dpp %{c}, %{n + c}, %{2 * n + l} row_newbcast:{off + l}{M}")
    outs = ", ".join(f'"+v"(acc[{c}])' for c in range(n))
    ins = ", ".join([f'"v"(b[{c}])' for c in range(n)] + [f'"v"(a[{l}])' for l in range(n)])
    body = "\\n\\t".join(lines)
    return (f"__device__ __forceinline__ void mst_rowmul_lt_{n}_{off}(double (&acc)[{n}], const double (&a)[{n}],"
            f" const double (&b)[{n}])\n{{\n    asm(\"{body}\"\n        : {outs}\n        : {ins});\n}}\n")


def mst_rowdot(n, off):
    # acc[c] (+|-)= bcast_{off+c}(b[m]) * a[m]: row r of A B' (lane off+c holds row c of B); operands acc, b, a
    out = []
    for sign, nm in (("", "mst_rowdot"), ("-", "mst_rowdot_neg")):
        lines = ["s_nop 1"]
        for m in range(n):
            for c in range(n):
                lines.append(f"v_fmac_f64_dpp %{c}, {sign}%{n + m}, %{2 * n + m} row_newbcast:{off + c}{M}")
        outs = ", ".join(f'"+v"(acc[{c}])' for c in range(n))
        ins = ", ".join([f'"v"(b[{m}])' for m in range(n)] + [f'"v"(a[{m}])' for m in range(n)])
        body = "\\n\\t".join(lines)
        out.append(f"__device__ __forceinline__ void {nm}_{n}_{off}(double (&acc)[{n}], const double (&a)[{n}],"
                   f" const double (&b)[{n}])\n{{\n    asm(\"{body}\"\n        : {outs}\n        : {ins});\n}}\n")
    return "\n".join(out)


def mst_chol(n, off):
    # right-looking row-distributed Cholesky, column j done: lr[jp] -= bcast_{off+jp}(lj) * lj for jp > j, then the
    # next pivot bcast_{off+j+1}(lr[j+1])
    out = []
    for j in range(n - 1):
        lines = ["s_nop 1"]
        ops = []
        for k, jp in enumerate(range(j + 1, n)):
            lines.append(f"v_fmac_f64_dpp %{k}, -%{n - j}, %{n - j} row_newbcast:{off + jp}{M}")
            ops.append(f'"+v"(lr[{jp}])')
        m = n - j - 1
        if m < 3:
            lines.append("s_nop 1")
        lines.append(f"v_mov_b64_dpp %{m}, %0 row_newbcast:{off + j + 1}{M}")
        outs = ", ".join(ops + ['"=&v"(piv)'])
        body = "\\n\\t".join(lines)
        out.append(f"__device__ __forceinline__ void mst_chol_{n}_{off}_{j}(double (&lr)[{n}], double lj, double& piv)\n"
                   f"{{\n    asm(\"{body}\"\n        : {outs}\n        : \"v\"(lj));\n}}\n")
    cases = "\n".join(f"    if constexpr (J == {j}) mst_chol_{n}_{off}_{j}(lr, lj, piv);" for j in range(n - 1))
    out.append(f"template <int J>\n__device__ __forceinline__ void mst_chol_{n}_{off}(double (&lr)[{n}], double lj,"
               f" double& piv)\n{{\n{cases}\n}}\n")
    return "\n".join(out)


def mst_trsv(n, off):
    # forward substitution y L' = u, y_j known: u[m] -= bcast_{off+m}(lc) * y for m > j (lc: the lane's L[.][j])
    out = []
    for j in range(n - 1):
        lines = ["s_nop 1"]
        ops = []
        for k, m in enumerate(range(j + 1, n)):
            lines.append(f"v_fmac_f64_dpp %{k}, -%{n - j - 1}, %{n - j} row_newbcast:{off + m}{M}")
            ops.append(f'"+v"(u[{m}])')
        outs = ", ".join(ops)
        body = "\\n\\t".join(lines)
        out.append(f"__device__ __forceinline__ void mst_trsv_{n}_{off}_{j}(double (&u)[{n}], double lc, double y)\n"
                   f"{{\n    asm(\"{body}\"\n        : {outs}\n        : \"v\"(lc), \"v\"(y));\n}}\n")
    cases = "\n".join(f"    if constexpr (J == {j}) mst_trsv_{n}_{off}_{j}(u, lc, y);" for j in range(n - 1))
    out.append(f"template <int J>\n__device__ __forceinline__ void mst_trsv_{n}_{off}(double (&u)[{n}], double lc,"
               f" double y)\n{{\n{cases}\n}}\n")
    return "\n".join(out)


def mst_vdot(n, off):
    # acc + sum_l bcast_{off+l}(x) * a[l] as two interleaved partial sums (x: a lane-distributed vector)
    lines = ["s_nop 1"]
    for l in range(n):
        lines.append(f"v_fmac_f64_dpp %{l % 2}, %2, %{3 + l} row_newbcast:{off + l}{M}")
    ins = ", ".join(['"v"(x)'] + [f'"v"(a[{l}])' for l in range(n)])
    body = "\\n\\t".join(lines)
    return (f"__device__ __forceinline__ double mst_vdot_{n}_{off}(double acc, double x, const double (&a)[{n}])\n{{\n"
            f"    double p1 = 0.0;\n    asm(\"{body}\"\n        : \"+v\"(acc), \"+v\"(p1)\n        : {ins});\n"
            f"    return acc + p1;\n}}\n")


def generate():
    parts = ["// team_asm_gen.hpp -- GENERATED by tools/gen_team_asm.py; do not edit.",
             "// Whole-block fused-DPP kernels of the team Riccati step (see the generator's docstring).",
             "#pragma once", "", "#include <hip/hip_runtime.h>", "", "namespace nmpc {", ""]
    for nx, nu in SHAPES:
        nv = nx + nu
        parts += [pg_block(nx, nu), mrow_pg_block(nx, nu)] + [mcol_var_block(nx, nu, g) for g in VAR_ROWS[(nx, nu)]]
        parts += [pg_block(nx, nu, "f32"), mcol_var_block(nx, nu, VAR_ROWS[(nx, nu)][0], "f32"),
                  chol_update(nx, nu, "f32")]
        parts += [chol_update(nx, nu),
                  dot_f32(nx, nu, f"dot_x_{nx}_{nu}"), dot_f32(nv, 0, f"dot_v_{nx}_{nu}"),
                  mst_rowmul(nx, nu), mst_rowmul_lt(nx, nu), mst_rowdot(nx, nu), mst_chol(nx, nu), mst_trsv(nx, nu), mst_vdot(nx, nu)]
    parts += ["}  // namespace nmpc", ""]
    return "\n".join(parts)


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else OUT
    with open(out, "w") as fh:
        fh.write(generate())
    print("wrote", out)


if __name__ == "__main__":
    main()
