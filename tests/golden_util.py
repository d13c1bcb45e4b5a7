"""Helpers to load the golden fixtures (tests/golden/*.npz, made by oracle/gen_golden.py from oracle/_ref)."""
import os

import numpy as np

import pyoracle as po

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name), allow_pickle=False))


def box_from(arr):
    b = po.OxBox()
    for k in range(6):
        b.lim[k] = float(arr[k])
    for k in range(3):
        b.bnd[k] = int(arr[6 + k])
    return b


def state_from(d, prefix):
    n = d[prefix + "x"].size
    st = po.HostState(n)
    for name, _ in po.STATE_FIELDS:
        if prefix + name in d:  # fixtures made before the avClean fields existed hold no dV*
            st.arrays[name][:] = d[prefix + name]
    sc = d[prefix + "scalars"]
    st.minDt, st.minDt_m1, st.ttot, st.minDtCourant, st.minDtRho = [float(v) for v in sc]
    return st
