#!/usr/bin/env python3
"""Extracts the reference's own mesh fixtures into tests/golden/ as plain data.

The reference's mesh scene (config/environment_mesh.yaml) loads
test/meshes/bookshelves.dae (and the repo also ships test/meshes/cabnite.dae).  This script
reads the COLLADA <float_array> of vertex positions and the <triangles> vertex indices of each
file and writes them, unscaled and in the file's own units, as

    tests/golden/meshes.npz : <name>_vertices (V x 3 float64), <name>_triangles (T x 3 int32)

plus the scene placement of environment_mesh.yaml (position, RPY orientation, scale) for the
bookshelves.  Only data is written: no text of the reference's files.  Run in this container,
where /root/reference exists:  python tools/extract_mesh.py
"""
from __future__ import annotations

import os
import sys
import xml.etree.ElementTree as ET

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/stomp_motion_planner"
OUT = os.path.join(ROOT, "tests", "golden", "meshes.npz")


def read_dae(path):
    root = ET.parse(path).getroot()
    ns = root.tag.split("}")[0].strip("{")
    q = lambda t: "{%s}%s" % (ns, t)  # noqa: E731
    verts, tris = [], []
    for geom in root.iter(q("geometry")):
        mesh = geom.find(q("mesh"))
        srcs = {s.get("id"): s for s in mesh.findall(q("source"))}
        vert_node = mesh.find(q("vertices"))
        pos_id = vert_node.find(q("input")).get("source").lstrip("#")
        arr = srcs[pos_id].find(q("float_array"))
        v = np.array([float(x) for x in arr.text.split()], np.float64).reshape(-1, 3)
        base = sum(len(x) for x in verts)
        verts.append(v)
        for t in mesh.findall(q("triangles")):
            inputs = t.findall(q("input"))
            stride = max(int(i.get("offset")) for i in inputs) + 1
            voff = [int(i.get("offset")) for i in inputs if i.get("semantic") == "VERTEX"][0]
            idx = np.array([int(x) for x in t.find(q("p")).text.split()], np.int64).reshape(-1, stride)
            tris.append(idx[:, voff].reshape(-1, 3) + base)
    return np.concatenate(verts), np.concatenate(tris).astype(np.int32)


def main():
    out = {}
    for name in ("bookshelves", "cabnite"):
        v, t = read_dae(os.path.join(REF, "test", "meshes", name + ".dae"))
        out[name + "_vertices"] = v
        out[name + "_triangles"] = t
        print(f"{name}: {len(v)} vertices, {len(t)} triangles")
    # environment_mesh.yaml, the bookshelves entry (frame /base_footprint)
    out["bookshelves_position"] = np.array([1.05, 0.7, 0.0])
    out["bookshelves_rpy"] = np.array([0.0, 0.0, -1.57])
    out["bookshelves_scale"] = np.array([0.031, 0.031, 0.031])
    np.savez_compressed(OUT, **out)
    print(OUT, os.path.getsize(OUT), "B")


if __name__ == "__main__":
    sys.exit(main())
