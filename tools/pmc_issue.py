"""Issue accounting from rocprofv3 PMC passes (tools/pmc_kernels.sh with ISSUE=1, summarised by
tools/pmc_summary.py --json): per kernel the VALU-busy fraction of the SIMDs' cycles, the model
check (v_exp / v_rcp / ... = 2 quad-cycles, every other VALU instruction 1: SQ_ACTIVE_INST_VALU),
and the LDS-busy fraction of the CUs' LDS pipes.  GRBM_GUI_ACTIVE and the SQ counters are summed
over the 8 XCDs; MI355X: 256 CUs x 4 SIMDs.
With the MFMA pass (SQ_INSTS_MFMA, SQ_VALU_MFMA_BUSY_CYCLES): the MFMA-busy fraction of the SIMDs'
cycles and the MFMA rate against the chip's dense fp32 MFMA peak (every MFMA on this path is
v_mfma_f32_16x16x4_f32 = 2*16*16*4 flops; the launch's duration from the same pass's kernel
trace, `dur_ns`).  With the wait pass: SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY shares
of the wave cycles and SQ_BUSY_CYCLES against the elapsed cycles.
usage: python tools/pmc_issue.py <summary.json> [--out derived.json]"""
import json
import sys

N_XCD, N_CU, N_SIMD = 8, 256, 1024
FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: dense fp32 (MFMA = vector) peak
MFMA_FLOPS = 2 * 16 * 16 * 4    # v_mfma_f32_16x16x4_f32
KEYS = ["fused4_kernel<10, 10, 10, 12, true, true, false, false, 2>", "fused4_kernel<10, 10, 10, 12, true, true, false, false, 1>",
        "fused4_kernel<10, 10, 10, 12, true, true, false, false>", "small6_kernel<true, true, false, false>",
        "v8_kernel<true, 2>",
        "fixed_bwd_kernel<2, 10, 10, 10, 12, true, true, 2>", "fixed_bwd_kernel<2, 10, 10, 10, 12, true, true, 1>",
        "sweep7_kernel<true>", "sweep7_kernel<false>", "kansum_kernel",
        "wide_layer_kernel<10, true, true, 8>", "wide_fwd4_kernel", "wide_fwd_kernel", "kuramoto_fwd_kernel",
        "kuramoto_fwd_lanes_kernel<28>",
        "fetode::kanrnn_fwd_kernel<1>", "fetode::kanrnn_bwd_kernel<12, 1>", "wide_ferro_bwd_kernel",
        "wide_kan_gx_kernel", "wide_kan_gw_kernel"]


def main():
    d = json.load(open(sys.argv[1]))
    out = {}
    for name, c in d.items():
        key = next((k for k in KEYS if k in name), None)
        if key is None:
            continue
        if "GRBM_GUI_ACTIVE" not in c:
            continue
        cyc = c["GRBM_GUI_ACTIVE"] / N_XCD
        r = out[key] = {"cycles": cyc}
        if "SQ_ACTIVE_INST_VALU" in c and "SQ_INSTS_VALU_TRANS_F32" in c:
            valu = 4 * c["SQ_ACTIVE_INST_VALU"]
            model = 4 * (2 * c["SQ_INSTS_VALU_TRANS_F32"] + (c["SQ_INSTS_VALU"] - c["SQ_INSTS_VALU_TRANS_F32"]))
            r.update({"valu_busy_frac": valu / (N_SIMD * cyc), "lds_busy_frac": 4 * c["SQ_ACTIVE_INST_LDS"] / (N_CU * cyc),
                      "valu_insts_per_wave": c["SQ_INSTS_VALU"] / c["SQ_WAVES"],
                      "trans_share": c["SQ_INSTS_VALU_TRANS_F32"] / c["SQ_INSTS_VALU"],
                      "issue_model_over_counter": model / valu})
        if "SQ_INSTS_MFMA" in c and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            r["mfma_per_launch"] = c["SQ_INSTS_MFMA"]
            r["mfma_busy_frac"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (N_SIMD * cyc)
            if c.get("dur_ns"):
                tf = c["SQ_INSTS_MFMA"] * MFMA_FLOPS / (c["dur_ns"] * 1e-9) / 1e12
                r.update({"mfma_tflops": tf, "mfma_frac_of_fp32_peak": tf / FP32_MFMA_PEAK_TFLOPS,
                          "dur_us_profiled": c["dur_ns"] / 1e3})
        if "SQ_WAIT_ANY" in c and "SQ_WAVE_CYCLES" in c:
            wc = c["SQ_WAVE_CYCLES"]
            r.update({"wait_any_share": c["SQ_WAIT_ANY"] / wc, "wait_inst_any_share": c.get("SQ_WAIT_INST_ANY", 0) / wc,
                      "active_inst_any_share": c.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                      "sq_busy_cycles_per_xcd_over_elapsed": c.get("SQ_BUSY_CYCLES", 0) / N_XCD / cyc})
    for k, v in out.items():
        print(f"{k[:60]:60s} " + "  ".join(f"{n} {x:.3g}" for n, x in v.items() if n != "cycles"))
    if "--out" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--out") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
