"""Issue accounting from one rocprofv3 PMC pass (tools/pmc_kernels.sh with ISSUE=1, summarised by
tools/pmc_summary.py --json): per kernel the VALU-busy fraction of the SIMDs' cycles, the model
check (v_exp / v_rcp / ... = 2 quad-cycles, every other VALU instruction 1: SQ_ACTIVE_INST_VALU),
and the LDS-busy fraction of the CUs' LDS pipes.  GRBM_GUI_ACTIVE and the SQ counters are summed
over the 8 XCDs; MI355X: 256 CUs x 4 SIMDs.
usage: python tools/pmc_issue.py <summary.json> [--out derived.json]"""
import json
import sys

N_XCD, N_CU, N_SIMD = 8, 256, 1024
KEYS = ["fused4_kernel<10, 10, 10, 12, true, true, false>", "small6_kernel<true, true>",
        "fixed_bwd_kernel<2, 10, 10, 10, 12, true, true, 2>", "wide_layer_kernel<10, true, true, 8>",
        "wide_fwd_kernel", "kuramoto_fwd_kernel", "fetode::kanrnn_fwd_kernel<1>", "fetode::kanrnn_bwd_kernel<12, 1>"]


def main():
    d = json.load(open(sys.argv[1]))
    out = {}
    for name, c in d.items():
        key = next((k for k in KEYS if k in name), None)
        if key is None:
            continue
        cyc = c["GRBM_GUI_ACTIVE"] / N_XCD
        valu = 4 * c["SQ_ACTIVE_INST_VALU"]
        model = 4 * (2 * c["SQ_INSTS_VALU_TRANS_F32"] + (c["SQ_INSTS_VALU"] - c["SQ_INSTS_VALU_TRANS_F32"]))
        out[key] = {"cycles": cyc, "valu_busy_frac": valu / (N_SIMD * cyc), "lds_busy_frac": 4 * c["SQ_ACTIVE_INST_LDS"] / (N_CU * cyc),
                    "valu_insts_per_wave": c["SQ_INSTS_VALU"] / c["SQ_WAVES"],
                    "trans_share": c["SQ_INSTS_VALU_TRANS_F32"] / c["SQ_INSTS_VALU"],
                    "issue_model_over_counter": model / valu}
    for k, v in out.items():
        print(f"{k[:52]:52s} VALU busy {v['valu_busy_frac']:.2f}  LDS busy {v['lds_busy_frac']:.2f}  "
              f"model/counter {v['issue_model_over_counter']:.3f}  trans {v['trans_share']:.2f}")
    if "--out" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--out") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
