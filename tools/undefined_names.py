"""Names a Python function reads that no enclosing scope, import or builtin defines (CPU,
no imports of the checked files): the staged GPU tests (tests/test_gpu_staged.py) and the
GPU-only tools never run in this container, so a missing import there would only show on a
GPU box.  Scope-aware over nested functions and comprehensions; a static approximation
(module-level names bound anywhere at the top level count as defined).

    python tools/undefined_names.py FILE.py ...   (prints FILE LINE NAME; exit 1 if any)
"""
import ast
import builtins
import sys

def bound_names(fn):
    local = set()
    args = fn.args
    for a in args.args + args.posonlyargs + args.kwonlyargs + ([args.vararg] if args.vararg else []) + ([args.kwarg] if args.kwarg else []):
        local.add(a.arg)
    body = fn.body if isinstance(fn.body, list) else [fn.body]
    stack = list(body)
    while stack:
        n = stack.pop()
        if isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
            local.add(n.name); continue  # don't descend
        if isinstance(n, ast.Lambda):
            continue
        if isinstance(n, ast.Name) and isinstance(n.ctx, (ast.Store, ast.Del)): local.add(n.id)
        elif isinstance(n, (ast.Import, ast.ImportFrom)):
            for a in n.names: local.add((a.asname or a.name).split('.')[0])
        elif isinstance(n, ast.ExceptHandler) and n.name: local.add(n.name)
        elif isinstance(n, (ast.Global, ast.Nonlocal)):
            local.update(n.names)
        stack.extend(ast.iter_child_nodes(n))
    return local

def visit(fn, env, path, probs):
    local = bound_names(fn) | env
    body = fn.body if isinstance(fn.body, list) else [fn.body]
    stack = list(body)
    # default args / decorators evaluated in enclosing scope: skip
    while stack:
        n = stack.pop()
        if isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef, ast.Lambda)):
            visit(n, local, path, probs); continue
        if isinstance(n, ast.ClassDef):
            continue
        if isinstance(n, (ast.ListComp, ast.SetComp, ast.GeneratorExp, ast.DictComp)):
            extra = set()
            for g in n.generators:
                for m in ast.walk(g.target):
                    if isinstance(m, ast.Name): extra.add(m.id)
            inner = local | extra
            for m in ast.walk(n):
                if isinstance(m, ast.Name) and isinstance(m.ctx, ast.Load) and m.id not in inner:
                    probs.add((m.lineno, m.id))
            continue
        if isinstance(n, ast.Name) and isinstance(n.ctx, ast.Load) and n.id not in local:
            probs.add((n.lineno, n.id))
        stack.extend(ast.iter_child_nodes(n))

def check(path):
    tree = ast.parse(open(path).read())
    mod = set(dir(builtins)) | {"__file__", "__name__"}
    for node in ast.walk(tree):
        if isinstance(node, (ast.Import, ast.ImportFrom)) and node in tree.body:
            for a in node.names: mod.add((a.asname or a.name).split('.')[0])
    for node in tree.body:
        for n in ast.walk(node):
            if isinstance(n, (ast.FunctionDef, ast.ClassDef)) and node is n: mod.add(n.name)
        if isinstance(node, (ast.FunctionDef, ast.ClassDef, ast.AsyncFunctionDef)): mod.add(node.name)
        if isinstance(node, (ast.Assign, ast.AnnAssign, ast.For, ast.With, ast.If, ast.Try)):
            for n in ast.walk(node):
                if isinstance(n, ast.Name) and isinstance(n.ctx, ast.Store): mod.add(n.id)
                if isinstance(n, (ast.Import, ast.ImportFrom)):
                    for a in n.names: mod.add((a.asname or a.name).split('.')[0])
    probs = set()
    for node in ast.walk(tree):
        if isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef)) and node in tree.body:
            visit(node, mod, path, probs)
        if isinstance(node, ast.ClassDef) and node in tree.body:
            for b in node.body:
                if isinstance(b, ast.FunctionDef): visit(b, mod | {x.name for x in node.body if isinstance(x, ast.FunctionDef)}, path, probs)
    return sorted(probs)


if __name__ == "__main__":
    bad = [(p, *x) for p in sys.argv[1:] for x in check(p)]
    for b in bad:
        print(*b)
    sys.exit(1 if bad else 0)
