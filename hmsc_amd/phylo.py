"""Phylogenetic trees for ``Hmsc(phyloTree=...)``.

The reference turns a tree into the species correlation matrix with
``ape::vcv.phylo(phyloTree, model="Brownian", corr=TRUE)`` and reorders it by the
species names (``R/Hmsc.R:504-509``).  ape is not part of the reference (an
unvendored dependency, ``DESCRIPTION``), so its published algorithm is restated:
under Brownian motion the covariance of tips i and j is the summed edge length from
the root to their most recent common ancestor, the variance of tip i its root-to-tip
length, and ``corr=TRUE`` scales to unit diagonal.  Pinned against the reference's own
``TD$m$C``, which ``data-raw/simulateTestData.R`` built from ``TD$phy`` this way
(``tests/test_host_phylo.py``).

A tree is an ape ``phylo``-shaped mapping -- ``edge`` (n_edges x 2, 1-based: tips
1..n, the root n + 1, internal nodes above), ``edge.length``, ``tip.label``, ``Nnode``
-- or a Newick string (``read_tree``).
"""
import re

import numpy as np


def read_tree(newick):
    """Parse a Newick string ("((a:1,b:1):0.5,c:1.5);") into the ape ``phylo`` layout
    (ape::read.tree's numbering: tips 1..n in order of appearance, the root n + 1, internal
    nodes numbered in preorder)."""
    s = newick.strip()
    if not s.endswith(";"):
        raise ValueError("read_tree: a Newick string ends with ';'")
    s = s[:-1]
    pos = 0

    def label_and_length():
        nonlocal pos
        m = re.compile(r"\s*([^:,();\s]*)\s*(?::\s*([-+0-9.eE]+))?\s*").match(s, pos)
        pos = m.end()
        return m.group(1), (float(m.group(2)) if m.group(2) is not None else None)

    def node():
        nonlocal pos
        while pos < len(s) and s[pos].isspace():
            pos += 1
        children = []
        if pos < len(s) and s[pos] == "(":
            pos += 1
            while True:
                children.append(node())
                while s[pos].isspace():
                    pos += 1
                if s[pos] == ",":
                    pos += 1
                    continue
                if s[pos] == ")":
                    pos += 1
                    break
                raise ValueError(f"read_tree: unexpected {s[pos]!r} at {pos}")
        lab, ln = label_and_length()
        return {"label": lab, "length": ln, "children": children}

    root = node()
    if pos != len(s):
        raise ValueError(f"read_tree: trailing text at {pos}")
    tips, internal = [], []

    def collect(nd):
        if nd["children"]:
            internal.append(nd)
            for c in nd["children"]:
                collect(c)
        else:
            tips.append(nd)

    collect(root)
    n = len(tips)
    num = {id(t): k + 1 for k, t in enumerate(tips)}
    num.update({id(v): n + 1 + k for k, v in enumerate(internal)})
    edge, length = [], []

    def edges(nd):
        for c in nd["children"]:
            edge.append((num[id(nd)], num[id(c)]))
            length.append(c["length"] if c["length"] is not None else np.nan)
            edges(c)

    edges(root)
    return {"edge": np.asarray(edge, dtype=np.int64), "edge.length": np.asarray(length, dtype=np.float64),
            "tip.label": [t["label"] for t in tips], "Nnode": len(internal)}


def _field(tree, name):
    try:
        return tree[name]
    except (KeyError, TypeError):
        return getattr(tree, name.replace(".", "_"))


def vcv_phylo(tree, corr=True):
    """ape::vcv.phylo(tree, model="Brownian", corr=corr): rows and columns in tip.label order.
    Returns (matrix, tip labels)."""
    if isinstance(tree, str):
        tree = read_tree(tree)
    edge = np.asarray(_field(tree, "edge"), dtype=np.int64)
    length = np.asarray(_field(tree, "edge.length"), dtype=np.float64)
    labels = [str(x) for x in _field(tree, "tip.label")]
    n = len(labels)
    if edge.ndim != 2 or edge.shape[1] != 2 or length.shape[0] != edge.shape[0]:
        raise ValueError("vcv_phylo: edge must be n_edges x 2 with one edge.length per edge")
    if np.any(~np.isfinite(length)):
        raise ValueError("vcv_phylo: the tree has no branch lengths")
    parent, plen = {}, {}
    for (a, b), ln in zip(edge, length):
        if b in parent:
            raise ValueError("vcv_phylo: a node has two parents")
        parent[int(b)], plen[int(b)] = int(a), float(ln)
    roots = {int(a) for a in edge[:, 0]} - set(parent)
    if len(roots) != 1:
        raise ValueError("vcv_phylo: the tree must have exactly one root")

    depth = {}

    def dep(v):  # summed edge length from the root
        path = []
        while v not in depth and v in parent:
            path.append(v)
            v = parent[v]
        d = depth.get(v, 0.0)
        for u in reversed(path):
            d += plen[u]
            depth[u] = d
        return depth.get(path[0], d) if path else d

    anc = []
    for i in range(1, n + 1):
        chain, v = [i], i
        while v in parent:
            v = parent[v]
            chain.append(v)
        anc.append(chain)
    V = np.empty((n, n))
    for i in range(n):
        si = set(anc[i])
        V[i, i] = dep(i + 1)
        for j in range(i):
            mrca = next(v for v in anc[j] if v in si)   # the first shared ancestor going up
            V[i, j] = V[j, i] = dep(mrca)
    if corr:
        d = np.sqrt(np.diag(V))
        V = V / d[:, None] / d[None, :]
    return V, labels
