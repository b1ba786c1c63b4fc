"""Per-call options map (`include/slate/types.hh:32-81, 211-271`).

``Options`` is a plain ``dict`` keyed by :class:`Option`; `get_option`
returns the typed value or a default, exactly like SLATE's
`get_option<T>(opts, key, default)`.  Values may also be given by string
name (``{"lookahead": 2}``) for convenience.
"""
from __future__ import annotations

import os

from .enums import (MethodCholQR, MethodEig, MethodGels, MethodGemm, MethodHemm,
                    MethodLU, MethodSVD, MethodTrsm, Option, Target)

Options = dict

_TYPES = {
    Option.Target: Target,
    Option.MethodCholQR: MethodCholQR,
    Option.MethodEig: MethodEig,
    Option.MethodGels: MethodGels,
    Option.MethodGemm: MethodGemm,
    Option.MethodHemm: MethodHemm,
    Option.MethodLU: MethodLU,
    Option.MethodTrsm: MethodTrsm,
    Option.MethodSVD: MethodSVD,
}

# Library-wide defaults.  Overridable with SLATE_AMD_<NAME> environment
# variables (e.g. SLATE_AMD_LOOKAHEAD=2), mirroring SLATE's env knobs.
DEFAULTS = {
    Option.Lookahead: 1,
    Option.InnerBlocking: 32,
    Option.MaxPanelThreads: 1,
    Option.HoldLocalWorkspace: False,
    Option.Depth: 2,
    Option.MaxIterations: 30,
    Option.UseFallbackSolver: True,
    Option.PivotThreshold: 1.0,
    Option.PrintVerbose: 4,
    Option.PrintEdgeItems: 16,
    Option.PrintWidth: 10,
    Option.PrintPrecision: 4,
    Option.UseGraph: False,
}


def _normalize_key(k):
    if isinstance(k, Option):
        return k
    if isinstance(k, str):
        norm = k.replace("_", "").lower()
        for o in Option:
            if o.name.lower() == norm:
                return o
    raise KeyError(f"unknown option {k!r}")


def normalize(opts) -> dict:
    if not opts:
        return {}
    out = {}
    for k, v in dict(opts).items():
        key = _normalize_key(k)
        t = _TYPES.get(key)
        if t is not None and not isinstance(v, t):
            v = t.from_string(v)
        out[key] = v
    return out


def get_option(opts, key: Option, default=None):
    opts = normalize(opts)
    if key in opts:
        return opts[key]
    env = os.environ.get("SLATE_AMD_" + key.name.upper())
    if env is not None:
        t = _TYPES.get(key)
        if t is not None:
            return t.from_string(env)
        if isinstance(default, bool):
            return env.lower() in ("1", "true", "yes", "y")
        if isinstance(default, int):
            return int(env)
        if isinstance(default, float):
            return float(env)
        return env
    if default is not None:
        return default
    return DEFAULTS.get(key)
