"""Hmsc(phyloTree=...) (R/Hmsc.R:504-509): the tree's Brownian correlation matrix
(ape::vcv.phylo restated, hmsc_amd/phylo.py) reordered by species names.  Pinned against
the reference's own TD$m, built from TD$phy this way: TD$m$C is the fixture's C (CPU only)."""
import numpy as np
import pytest

import hmsc_amd as H
from hmsc_amd.phylo import read_tree, vcv_phylo
from test_golden_td import D, M, td_model


def td_tree():
    return {"edge": D["phy_edge"], "edge.length": D["phy_edge_length"], "tip.label": M["phy_tip_label"],
            "Nnode": M["phy_Nnode"]}


def test_vcv_phylo_reproduces_td_m_C():
    V, tips = vcv_phylo(td_tree(), corr=True)
    ix = [tips.index(s) for s in M["spNames"]]
    np.testing.assert_allclose(V[np.ix_(ix, ix)], D["C"], rtol=0, atol=1e-15)


def test_hmsc_with_phylo_tree_equals_td_m():
    """TD$m rebuilt with phyloTree = TD$phy instead of C: the same C, and the tree kept."""
    hM0 = td_model()
    kw = dict(Y=D["Y"], XData=hM0.XData, XFormula="~x1+x2", TrData=hM0.TrData, TrFormula="~T1+T2",
              ranLevels={"sample": hM0.ranLevels["sample"], "plot": hM0.ranLevels["plot"]},
              studyDesign=hM0.studyDesign, distr="probit", spNames=M["spNames"])
    hM = H.Hmsc(phyloTree=td_tree(), **kw)
    np.testing.assert_allclose(hM.C, D["C"], rtol=0, atol=1e-15)
    assert hM.phyloTree is not None
    with pytest.raises(ValueError, match="at maximum one"):
        H.Hmsc(phyloTree=td_tree(), C=D["C"], **kw)


def test_newick_round_trip():
    """A Newick string gives ape's numbering (tips in order, root n + 1) and the same matrix as
    the explicit edge table; covariances are root-to-MRCA path lengths."""
    t = read_tree("((a:1,b:2):0.5,(c:1.5,d:1.5):1);")
    assert t["tip.label"] == ["a", "b", "c", "d"] and t["Nnode"] == 3
    assert t["edge"][0].tolist() == [5, 6]
    V, tips = vcv_phylo(t, corr=False)
    np.testing.assert_allclose(np.diag(V), [1.5, 2.5, 2.5, 2.5])
    assert V[0, 1] == 0.5 and V[2, 3] == 1.0 and V[0, 2] == 0.0
    C, _ = vcv_phylo("((a:1,b:2):0.5,(c:1.5,d:1.5):1);")
    np.testing.assert_allclose(C, V / np.sqrt(np.outer(np.diag(V), np.diag(V))))
    # the TD tree written as Newick
    V2, tips2 = vcv_phylo("((sp_003:0.26276183,sp_004:0.26276183):1.00593144,"
                          "(sp_001:0.12217261,sp_002:0.12217261):1.14652066);")
    V1, tips1 = vcv_phylo(td_tree())
    assert tips1 == tips2
    np.testing.assert_allclose(V2, V1, rtol=1e-7)
