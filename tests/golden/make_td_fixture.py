"""Generate the committed TD golden fixtures from the reference's ``data/TD.rda``.

Run once in the build container (``/root/reference`` exists only there):

    python tests/golden/make_td_fixture.py

Outputs (data only — inputs and expected outputs, no reference source):
  * ``td.npz``       — TD inputs (Y, X model matrix, XScaled, Tr, TrScaled, C, Pi,
                       xycoords, scaling parameters, priors, rhopw, alphapw) and the
                       fitted ``TD$m$postList`` (2 chains x 100 samples, all fields).
  * ``td_meta.json`` — names (species / covariates / traits / levels), dims, and
                       the deterministic known answers the reference's own tests
                       assert (tests/testthat/test-initialParameters.R:137-186,
                       test-WAIC.R:4, test-sampling.R:164-169).
TD$m was fitted by ``data-raw/simulateTestData.R:70`` with
``sampleMcmc(thin=1, samples=100, transient=50, nChains=2)``.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from rdata import read_rda  # noqa: E402

REF = "/root/reference/data/TD.rda"


def arr(o):
    return None if o is None else np.asarray(o.array(), dtype=np.float64)


def main():
    TD = read_rda(REF)["TD"]
    m = TD["m"]
    out = {}
    out["Y"] = arr(m["Y"])
    out["YScaled"] = arr(m["YScaled"])
    out["X"] = arr(m["X"])
    out["XScaled"] = arr(m["XScaled"])
    out["XScalePar"] = arr(m["XScalePar"])
    out["Tr"] = arr(m["Tr"])
    out["TrScaled"] = arr(m["TrScaled"])
    out["TrScalePar"] = arr(m["TrScalePar"])
    out["C"] = arr(m["C"])
    out["Pi"] = arr(m["Pi"]).astype(np.int64)
    out["distr"] = arr(m["distr"])
    out["V0"] = arr(m["V0"])
    out["f0"] = arr(m["f0"])
    out["mGamma"] = arr(m["mGamma"])
    out["UGamma"] = arr(m["UGamma"])
    out["aSigma"] = arr(m["aSigma"])
    out["bSigma"] = arr(m["bSigma"])
    out["rhopw"] = arr(m["rhopw"])
    # TD$m was built with phyloTree = TD$phy (R/Hmsc.R:504-509 makes TD$m$C from it)
    phy = m["phyloTree"]
    out["phy_edge"] = arr(phy["edge"]).astype(np.int64)
    out["phy_edge_length"] = arr(phy["edge.length"])
    out["xycoords"] = arr(TD["xycoords"])
    out["x1"] = arr(TD["X"]["x1"])
    rl = m["rL"]
    rl_meta = []
    for r, name in enumerate(rl.names()):
        lv = rl.value[r]
        d = {"name": name}
        for k in ("sDim", "xDim", "nu", "a1", "b1", "a2", "b2", "nfMax", "nfMin", "N"):
            v = lv[k]
            d[k] = None if v is None else float(np.asarray(v.value).ravel()[0])
        sm = lv["spatialMethod"]
        d["spatialMethod"] = None if sm is None else sm.value[0]
        if lv["alphapw"] is not None:
            out[f"alphapw_{r}"] = arr(lv["alphapw"])
        if lv["s"] is not None:
            out[f"s_{r}"] = arr(lv["s"])
        rl_meta.append(d)

    post = m["postList"]
    n_chains = len(post.value)
    n_samp = len(post.value[0].value)
    fields = post.value[0].value[0].names()
    for c in range(n_chains):
        for f in ("Beta", "Gamma", "V", "rho", "sigma"):
            out[f"post_{f}_c{c}"] = np.stack([arr(s[f]) for s in post.value[c].value])
        for f in ("Eta", "Lambda", "Alpha", "Psi", "Delta"):
            for r in range(len(rl_meta)):
                out[f"post_{f}{r}_c{c}"] = np.stack(
                    [np.asarray(arr(s[f].value[r])) for s in post.value[c].value])

    sd = m["studyDesign"]
    meta = {
        "source": "reference data/TD.rda (TD$m, fitted by data-raw/simulateTestData.R:70)",
        "ny": int(m["ny"].value[0]), "ns": int(m["ns"].value[0]), "nc": int(m["nc"].value[0]),
        "nt": int(m["nt"].value[0]), "nr": int(m["nr"].value[0]),
        "np": [int(x) for x in m["np"].value],
        "spNames": list(m["spNames"].value), "covNames": list(m["covNames"].value),
        "trNames": list(m["trNames"].value), "rLNames": list(m["rLNames"].value),
        "XInterceptInd": int(m["XInterceptInd"].value[0]),
        "TrInterceptInd": int(m["TrInterceptInd"].value[0]),
        "studyDesign_plot": [int(x) for x in sd["plot"].value],
        "studyDesign_plot_levels": list(sd["plot"].attr["levels"].value),
        "n_hM_fields": len(m.names()),
        "hM_fields": m.names(),
        "postList_fields": fields,
        "n_chains": n_chains, "n_samples": n_samp,
        "samples": int(m["samples"].value[0]), "transient": int(m["transient"].value[0]),
        "thin": int(m["thin"].value[0]),
        "rL": rl_meta,
        "phy_tip_label": list(phy["tip.label"].value), "phy_Nnode": int(phy["Nnode"].value[0]),
        # known answers from the reference's own tests
        "known": {
            "sum_detQg_round": -68, "sum_Qg_round": 575, "sum_iQg_round": 293, "sum_RQg_round": 461,
            "sum_detWg_round": -601, "sum_Wg_round": 4620, "sum_iWg_round": 329, "sum_RiWg_round": 476,
            "WAIC_round1": 0.8, "len_hM_after_sampling": 72, "len_postList_sample": 13,
        },
    }
    np.savez_compressed(os.path.join(HERE, "td.npz"), **{k: v for k, v in out.items() if v is not None})
    with open(os.path.join(HERE, "td_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote td.npz with", len(out), "arrays;", n_chains, "chains x", n_samp, "samples")


if __name__ == "__main__":
    main()
