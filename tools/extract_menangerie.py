"""Extract the Relay programs of the reference's own float test models (mnist, resnet50,
mobilenet) and the constant shapes their metadata tables list, from
/root/reference/tests/python/relay/collage/menangerie.py (read as text with ``ast``: nothing of
the reference is imported or run).  Writes, per model, tests/golden/menangerie_<name>.relay (the
program string as the reference hands it to tvm.parser.parse) and
tests/golden/menangerie_<name>.json (input name/shape and the ``meta[relay.Constant][i]`` shapes).
The constants' values are regenerated from a seed by the tests (the reference draws them with
np.random.rand at test time, menangerie.py:65-70).

    python tools/extract_menangerie.py [path/to/menangerie.py]
"""
import ast
import json
import os
import sys

MODELS = {"mnist": "mnist_consts", "resnet50": "resnet50_consts", "mobilenet": "mobilenet_consts"}
SRC = "/root/reference/tests/python/relay/collage/menangerie.py"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


def _functions(tree):
    return {n.name: n for n in tree.body if isinstance(n, ast.FunctionDef)}


def _program(fn: ast.FunctionDef) -> str:
    for node in ast.walk(fn):
        if isinstance(node, ast.Call) and getattr(node.func, "attr", "") == "parse":
            arg = node.args[0]
            if isinstance(arg, ast.Constant) and isinstance(arg.value, str):
                return arg.value
    raise ValueError(f"{fn.name}: no tvm.parser.parse(<string>) call")


def _const_shapes(fn: ast.FunctionDef):
    for node in ast.walk(fn):
        if isinstance(node, ast.Call) and getattr(node.func, "id", "") == "make_consts":
            return [list(t) for t in ast.literal_eval(node.args[1])]
    raise ValueError(f"{fn.name}: no make_consts(dtype, [shapes]) call")


def _inputs(fn: ast.FunctionDef):
    for node in ast.walk(fn):
        if isinstance(node, ast.Dict):
            keys = [k.value for k in node.keys if isinstance(k, ast.Constant)]
            if "input_shapes" in keys:
                shapes = ast.literal_eval(node.values[keys.index("input_shapes")])
                return {k: list(v) for k, v in shapes.items()}
    raise ValueError(f"{fn.name}: no input_shapes")


def main(src: str = SRC) -> None:
    with open(src) as f:
        tree = ast.parse(f.read())
    fns = _functions(tree)
    os.makedirs(OUT, exist_ok=True)
    for name, consts in MODELS.items():
        text = _program(fns[name])
        meta = {"model": name, "source": "tests/python/relay/collage/menangerie.py", "function": name,
                "inputs": _inputs(fns[name]), "constant_shapes": _const_shapes(fns[consts]),
                "constant_dtype": "float32"}
        with open(os.path.join(OUT, f"menangerie_{name}.relay"), "w") as f:
            f.write(text.strip() + "\n")
        with open(os.path.join(OUT, f"menangerie_{name}.json"), "w") as f:
            json.dump(meta, f, indent=1)
        print(f"{name}: {len(text.splitlines())} lines, {len(meta['constant_shapes'])} constants")


if __name__ == "__main__":
    main(*sys.argv[1:])
