"""Record the drop-in boundary: every intra-package import the reference makes.

Run only in the development container (the reference is not on the GPU box):

    python /root/repo/tests/golden/make_boundary_names.py [/root/reference]

The reference sources are PARSED with `ast` (read as text, nothing executed) and every
`from <src module> import ...` statement of every module under `src/` is written to
tests/golden/boundary_names.json, resolved to an absolute module name:

    {"replaced": [...modules this package ships...],
     "modules": {"src/client/federated_trainer.py": {"module": "src.client.federated_trainer",
                  "imports": [["src.shared.models", ["ClientCapabilities", ...]], ...],
                  "lazy_imports": [...imports inside functions...]}, ...},
     "required": {"src.shared.models": [names any caller imports from it], ...}}

tests/test_boundary_cpu.py checks that (1) every name in "required" for a replaced module
resolves in this package's module, and (2) a stub tree of the non-replaced reference modules
(the same import statements, stub definitions for the names others import from them) placed
behind this package on sys.path imports cleanly: the replaced modules come from here, the
rest from the other tree (pkgutil.extend_path in src/__init__.py and its subpackages).
"""
from __future__ import annotations

import ast
import json
import os
import sys

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "boundary_names.json")
PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                   "federated-learning-for-privacy-preserving-image-classification_amd")


def module_name(rel_path: str) -> str:
    parts = rel_path[:-3].split(os.sep)
    if parts[-1] == "__init__":
        parts = parts[:-1]
    return ".".join(parts)


def resolve(current: str, is_pkg: bool, node: ast.ImportFrom) -> str | None:
    if node.level == 0:
        return node.module if node.module and node.module.split(".")[0] == "src" else None
    base = current.split(".")
    if not is_pkg:
        base = base[:-1]
    base = base[: len(base) - (node.level - 1)]
    return ".".join(base + ([node.module] if node.module else []))


def replaced_modules() -> list[str]:
    out = []
    root = os.path.join(PKG, "src")
    for dp, _, files in os.walk(root):
        for f in files:
            if f.endswith(".py") and f != "__init__.py":
                rel = os.path.relpath(os.path.join(dp, f), PKG)
                out.append(module_name(rel))
    return sorted(out)


def main(ref: str) -> None:
    replaced = replaced_modules()
    modules, required = {}, {}
    src = os.path.join(ref, "src")
    for dp, _, files in sorted(os.walk(src)):
        for f in sorted(files):
            if not f.endswith(".py"):
                continue
            path = os.path.join(dp, f)
            rel = os.path.relpath(path, ref)
            mod = module_name(rel)
            with open(path, encoding="utf-8") as fh:
                try:
                    tree = ast.parse(fh.read(), filename=rel)
                except SyntaxError as e:  # grpc_server.py:582 does not parse in py3.10
                    modules[rel] = {"module": mod, "syntax_error": f"line {e.lineno}",
                                    "imports": []}
                    tree = None
            if tree is None:
                # fall back to the import block only (the statements before the first def)
                with open(path, encoding="utf-8") as fh:
                    lines = fh.read().splitlines()
                head = []
                for ln in lines:
                    if ln.startswith(("def ", "class ", "@")):
                        break
                    head.append(ln)
                tree = ast.parse("\n".join(head))
            top = set()  # module-level statements (incl. inside module-level try / if)
            stack = list(tree.body)
            while stack:
                node = stack.pop()
                top.add(id(node))
                if isinstance(node, (ast.Try, ast.If)):
                    stack.extend(node.body + node.orelse
                                 + [h for hd in getattr(node, "handlers", []) for h in hd.body])
            imps, lazy = [], []
            for node in ast.walk(tree):
                if isinstance(node, ast.ImportFrom):
                    target = resolve(mod, f == "__init__.py", node)
                    if target is None:
                        continue
                    names = [a.name for a in node.names]
                    (imps if id(node) in top else lazy).append([target, names])
                    if mod not in replaced:
                        required.setdefault(target, set()).update(names)
            ent = modules.setdefault(rel, {"module": mod})
            ent["imports"], ent["lazy_imports"] = imps, lazy
    out = {"generated_from": "reference src/ (ast, not executed)",
           "replaced": replaced,
           "modules": modules,
           "required": {k: sorted(v) for k, v in sorted(required.items())}}
    with open(OUT, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print(f"wrote {OUT}: {len(modules)} modules, "
          f"{sum(len(v) for v in out['required'].values())} required names")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
