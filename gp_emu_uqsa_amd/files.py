"""Config and beliefs files: the reference's text-file surface.

Format (README.md:158-314 of the reference): one ``key value`` per line, split
at the first space; unknown keys are ignored.  Bounds and ``input_minmax`` are
Python list expressions.  The reference ``eval``s them in a module that imported
numpy as np (_emulatorclasses.py:76-78, :95, :211), so a file may hold arithmetic
(``[[0.1, 2*0.5]]``), numpy constants (``np.pi``) and the ``np.float64(x)``
spellings that NumPy 2 makes the reference write into updated beliefs files
(SURVEY.md Appendix A).  Here they go through ``literal``: a restricted evaluator
of the expression tree that computes exactly those forms -- numbers, lists /
tuples, + - * / // % **, unary +/-, np.pi / np.e / np.inf / np.nan, and the numpy
scalar constructors and elementary functions (float64, sqrt, exp, log, ...) -- and
refuses anything else (names, attributes, other calls) with a ValueError instead
of executing it.  That refusal is the one deliberate difference from ``eval``.
Error behaviour otherwise follows the reference: a message, then ``SystemExit``.
"""
from __future__ import annotations

import ast
import math
import operator


CONFIG_REQUIRED = ("beliefs", "inputs", "outputs", "tv_config", "delta_bounds", "nugget_bounds",
                   "sigma_bounds", "tries", "constraints")
BELIEFS_REQUIRED = ("active", "output", "basis_str", "basis_inf", "beta", "delta", "sigma", "nugget",
                    "fix_nugget", "mucm")


def _die(msg):
    print(msg)
    raise SystemExit(1)


_BINOPS = {ast.Add: operator.add, ast.Sub: operator.sub, ast.Mult: operator.mul, ast.Div: operator.truediv,
           ast.FloorDiv: operator.floordiv, ast.Mod: operator.mod, ast.Pow: operator.pow}
_UNOPS = {ast.USub: operator.neg, ast.UAdd: operator.pos}
_NP_CONST = {"pi": math.pi, "e": math.e, "inf": math.inf, "nan": math.nan}
_NP_FUNCS = {"float64": float, "float32": float, "float_": float, "int64": int, "int32": int, "int_": int,
             "sqrt": math.sqrt, "exp": math.exp, "log": math.log, "log10": math.log10, "abs": abs,
             "fabs": math.fabs}
_NP_NAMES = ("np", "numpy", "_np")


def _np_member(node, table):
    if (isinstance(node, ast.Attribute) and isinstance(node.value, ast.Name)
            and node.value.id in _NP_NAMES and node.attr in table):
        return table[node.attr]
    raise ValueError(f"unsupported expression in a list value: {ast.dump(node)}")


def _evaluate(node):
    if isinstance(node, ast.Expression):
        return _evaluate(node.body)
    if isinstance(node, ast.Constant) and isinstance(node.value, (int, float)) and not isinstance(node.value, bool):
        return node.value
    if isinstance(node, ast.List):
        return [_evaluate(e) for e in node.elts]
    if isinstance(node, ast.Tuple):
        return tuple(_evaluate(e) for e in node.elts)
    if isinstance(node, ast.BinOp) and type(node.op) in _BINOPS:
        return _BINOPS[type(node.op)](_evaluate(node.left), _evaluate(node.right))
    if isinstance(node, ast.UnaryOp) and type(node.op) in _UNOPS:
        return _UNOPS[type(node.op)](_evaluate(node.operand))
    if isinstance(node, ast.Attribute):
        return _np_member(node, _NP_CONST)
    if isinstance(node, ast.Call) and not node.keywords:
        fn = _np_member(node.func, _NP_FUNCS)
        return fn(*[_evaluate(a) for a in node.args])
    raise ValueError(f"unsupported expression in a list value: {ast.dump(node)}")


def literal(text: str):
    """The reference's eval() of a list value (_emulatorclasses.py:76-78, :211),
    restricted to numbers and arithmetic (see the module docstring)."""
    return _evaluate(ast.parse(text.strip(), mode="eval"))


def read_key_values(path: str, missing_value_exits: bool) -> dict:
    """Read ``key value`` lines.  A line without a space raises ValueError in the
    reference; Beliefs catches it (message + exit), Config does not."""
    table = {}
    try:
        with open(path, "r") as fh:
            for line in fh:
                try:
                    key, val = line.split(" ", 1)
                except ValueError:
                    if missing_value_exits:
                        _die("ERROR: Some specifications seem to be missing values.")
                    raise
                table[key] = val
    except OSError:
        _die("ERROR: Problem reading file.")
    return table


class Config:
    """Configuration file (reference: _emulatorclasses.py:32-98)."""

    def __init__(self, config_file):
        self.config_file = config_file
        print("*** Reading config file:", config_file, "***")
        self.config = read_key_values(config_file, missing_value_exits=False)
        for key in CONFIG_REQUIRED:
            if key not in self.config:
                print('WARNING: "', key, '" specification is missing')
                raise SystemExit(1)
        self._parse()

    def _parse(self):
        c = self.config
        self.beliefs = str(c["beliefs"]).strip()
        self.inputs = str(c["inputs"]).strip()
        self.outputs = str(c["outputs"]).strip()
        tv = [int(v) for v in str(c["tv_config"]).strip().split(" ")]
        self.tv_config = tv
        if len(tv) != 3:
            _die("WARNING: tv_config requires 3 entries.")
        print("T-V config:", self.tv_config)
        self.delta_bounds = literal(c["delta_bounds"])
        self.nugget_bounds = literal(c["nugget_bounds"])
        self.sigma_bounds = literal(c["sigma_bounds"])
        self.bounds = tuple(self.delta_bounds + self.nugget_bounds + self.sigma_bounds)
        self.tries = int(str(c["tries"]).strip())
        print("number of tries for optimum:", self.tries)
        cons = str(c["constraints"]).strip()
        if cons in ("none", "bounds"):
            self.constraints = cons
        else:
            self.constraints = "standard"
            if cons != "standard":
                print("unrecognised constraints option, defaulting")
        print("constraints:", self.constraints)
        if "fix" in c:
            self.fix = literal(c["fix"])
            print("Fixing hyperparameters:", self.fix)
        else:
            self.fix = []


def _ints_or_all(text):
    toks = str(text).strip().split(" ")
    return [] if toks[0] == "all" else [int(t) for t in toks]


class Beliefs:
    """Beliefs file (reference: _emulatorclasses.py:102-250)."""

    def __init__(self, beliefs_file):
        self.beliefs_file = beliefs_file
        print("\n*** Reading beliefs file:", beliefs_file, "***")
        self.beliefs = read_key_values(beliefs_file, missing_value_exits=True)
        for key in BELIEFS_REQUIRED:
            if key not in self.beliefs:
                print('WARNING: "', key, '" specification is missing')
                raise SystemExit(1)
        self._parse()

    def _parse(self):
        b = self.beliefs
        if "active_index" in b:
            try:
                self.active_index = _ints_or_all(b["active_index"])
            except ValueError:
                print("WARNING: active_index should be 'all' or whitespaced integers,"
                      " setting value to 'unknown' and continuing")
                self.active_index = "unknown"
        self.active = _ints_or_all(b["active"])
        print("active:", self.active)
        if "output_index" in b:
            try:
                self.output_index = int(str(b["output_index"]).strip().split(" ")[0])
            except ValueError:
                print("WARNING: output_index should be an integer,"
                      " setting value to 'unknown' and continuing")
                self.output_index = "unknown"
        self.output = int(str(b["output"]).strip().split(" ")[0])
        print("output:", self.output)
        self.basis_str = str(b["basis_str"]).strip().split(" ")
        self.basis_inf = [int(v) for v in str(b["basis_inf"]).strip().split(" ")[1:]]
        self.beta = [float(v) for v in str(b["beta"]).strip().split(" ")]
        if len(self.basis_str) != len(self.basis_inf) + 1:
            _die("WARNING: basis_str & basis_inf need an equal number of "
                 "entires, including redundant first entry of basis_inf.")
        if len(self.basis_str) != len(self.beta):
            _die("WARNING: basis_str & beta need an equal number of entries.")
        self.delta = [float(v) for v in str(b["delta"]).strip().split(" ")]
        self.sigma = float(str(b["sigma"]).strip().split(" ")[0])
        self.nugget = float(str(b["nugget"]).strip().split(" ")[0])
        self.fix_nugget = str(b["fix_nugget"]).strip().split(" ")[0]
        self.alt_nugget = str(b["alt_nugget"]).strip().split(" ")[0] if "alt_nugget" in b else "F"
        self.mucm = str(b["mucm"]).strip().split(" ")[0]
        if self.mucm == "T" and self.alt_nugget == "T":
            _die("WARNING: mucm T cannot be used with alt_nugget T")
        self.input_minmax = literal(b["input_minmax"]) if "input_minmax" in b else []

    def final_beliefs(self, E, final=False):
        """Write the updated beliefs '<beliefs>-N[f]' (reference :217-250).
        input_minmax is written with plain floats (the reference's NumPy-2
        output writes np.float64(...) reprs; both forms are read back)."""
        suffix = "f" if final else ""
        filename = E.config.beliefs + "-" + str(E.tv_conf.no_of_trains) + suffix
        print("New beliefs to file", filename)
        ndelta = len(E.par.delta)
        idx = " ".join(str(i) for i in range(ndelta))
        lines = [
            "active_index " + (idx if self.active == [] else " ".join(map(str, self.active))),
            "active " + idx,
            "output_index " + str(self.output),
            "output 0 ",
            "basis_str " + " ".join(map(str, self.basis_str)),
            "basis_inf NA " + " ".join(map(str, self.basis_inf)),
            "beta " + " ".join(str(float(v)) for v in E.par.beta),
            "delta " + " ".join(str(float(v)) for v in list(E.par.delta)),
            "sigma " + str(float(E.par.sigma)),
            "nugget " + str(float(E.par.nugget)),
            "fix_nugget " + str(self.fix_nugget),
            "alt_nugget " + str(self.alt_nugget),
            "mucm " + str(self.mucm),
            "input_minmax " + str([[float(a), float(b)] for a, b in E.all_data.input_minmax]),
        ]
        try:
            with open(filename, "w") as fh:
                fh.write("\n".join(lines) + "\n")
        except OSError:
            _die("ERROR: Problem writing to file.")
