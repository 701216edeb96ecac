"""Transcribes the reference's DataEmbeddingLayer known answers into tests/golden/embedding_known_answers.json.

Source (read as text, never imported or executed): /root/reference/tests/data/test_data_embedding_layer.py
  test_joint_embeds  (:255-346)  JOINT bags with identity tables, with and without measurement-index normalisation
  test_split_embeds  (:348-576)  SPLIT bags (cat table I, cat_proj 0.5 I, num table 2 I, num_proj -I)
  test_forward       (:732-913)  the full forward on a 2-subject batch, static DROP / SUM_ALL

The file's `cases = [...]` literals (and `valid_params` / `default_batch`) are parsed with `ast` and evaluated by a
tiny literal evaluator below (numbers, lists, dicts incl. `**` merges, arithmetic on numbers, the torch tensor
constructors as typed lists, `StaticEmbeddingMode.X` as its string value, `PytorchBatch(**fields)` as a dict).
Nothing from the reference is executed. Run in this container only: python tests/golden/make_embedding_known_answers.py
"""
import ast
import json
import os
import sys

SRC = "/root/reference/tests/data/test_data_embedding_layer.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "embedding_known_answers.json")
_TENSORS = {"Tensor": "float32", "FloatTensor": "float32", "LongTensor": "int64", "BoolTensor": "bool"}


class Literal:
    def __init__(self, env):
        self.env = env

    def __call__(self, n):
        if isinstance(n, ast.Constant):
            return n.value
        if isinstance(n, (ast.List, ast.Tuple)):
            return [self(e) for e in n.elts]
        if isinstance(n, ast.Dict):
            out = {}
            for k, v in zip(n.keys, n.values):
                if k is None:
                    out.update(self(v))
                else:
                    out[self(k)] = self(v)
            return out
        if isinstance(n, ast.UnaryOp) and isinstance(n.op, ast.USub):
            return -self(n.operand)
        if isinstance(n, ast.BinOp):
            a, b = self(n.left), self(n.right)
            ops = {ast.Div: lambda: a / b, ast.Mult: lambda: a * b, ast.Add: lambda: a + b, ast.Sub: lambda: a - b}
            return ops[type(n.op)]()
        if isinstance(n, ast.Name):
            return self.env[n.id]
        if isinstance(n, ast.Attribute) and isinstance(n.value, ast.Name) and n.value.id == "StaticEmbeddingMode":
            return n.attr.lower()
        if isinstance(n, ast.Call):
            f = n.func
            if isinstance(f, ast.Attribute) and isinstance(f.value, ast.Name) and f.value.id == "torch":
                if f.attr in _TENSORS:
                    return {"dtype": _TENSORS[f.attr], "data": self(n.args[0])}
                if f.attr == "eye":
                    return {"eye": self(n.args[0])}
            if isinstance(f, ast.Name) and f.id == "PytorchBatch":
                return {"PytorchBatch": {kw.arg: self(kw.value) for kw in n.keywords}}
        raise ValueError(f"unsupported literal at line {getattr(n, 'lineno', '?')}: {ast.dump(n)[:120]}")


def _assignments(fn: ast.FunctionDef, env: dict):
    """Evaluates the function's top-level `name = <literal>` assignments in order."""
    out = {}
    for st in fn.body:
        if isinstance(st, ast.Assign) and len(st.targets) == 1 and isinstance(st.targets[0], ast.Name):
            name = st.targets[0].id
            try:
                out[name] = Literal({**env, **out})(st.value)
            except (ValueError, KeyError):
                continue
    return out


def main():
    tree = ast.parse(open(SRC).read())
    fns = {n.name: n for n in ast.walk(tree) if isinstance(n, ast.FunctionDef)}
    res = {"source": "tests/data/test_data_embedding_layer.py (reference), transcribed by "
                     "tests/golden/make_embedding_known_answers.py", "cases": []}
    spans = {"test_joint_embeds": "joint", "test_split_embeds": "split", "test_forward": "forward"}
    for fname, kind in spans.items():
        fn = fns[fname]
        vals = _assignments(fn, {})
        for c in vals["cases"]:
            c = dict(c)
            c["kind"] = kind
            c["ref_lines"] = f"{fn.lineno}-{fn.end_lineno}"
            res["cases"].append(c)
    json.dump(res, open(OUT, "w"), indent=1)
    print(f"wrote {len(res['cases'])} cases to {OUT}")


if __name__ == "__main__":
    sys.exit(main())
