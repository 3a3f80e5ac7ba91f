"""Static check for names a function reads that nothing defines.

No linter ships in the image, and a missing import inside a rarely-run path
(``cli serve``'s engine builder once read ``torch`` without importing it)
only shows up on the GPU box.  This walks every module's AST with a scope
model close enough for this code base: module globals (imports, defs,
classes, assignments, star-free), function parameters and locals, enclosing
function scopes, comprehension targets, ``global`` / ``nonlocal``, class
bodies (visible only to themselves), ``except ... as``, ``with ... as``,
walrus targets and builtins.

    python scripts/check_names.py [paths...]      # exit 1 on findings
"""
from __future__ import annotations

import ast
import builtins
import sys
from pathlib import Path
from typing import Iterable, List, Set, Tuple

BUILTINS = set(dir(builtins)) | {"__file__", "__name__", "__doc__", "__spec__", "__path__", "__builtins__",
                                 "__package__", "__loader__", "__class__", "__annotations__", "__qualname__",
                                 "__module__", "__dict__"}


def _targets(node: ast.AST) -> Iterable[str]:
    if isinstance(node, ast.Name):
        yield node.id
    elif isinstance(node, (ast.Tuple, ast.List)):
        for e in node.elts:
            yield from _targets(e)
    elif isinstance(node, ast.Starred):
        yield from _targets(node.value)


def _bound_in(body: List[ast.stmt], args: ast.arguments = None) -> Set[str]:
    """Names bound directly in a scope (not inside nested defs / classes)."""
    out: Set[str] = set()
    if args is not None:
        for a in args.posonlyargs + args.args + args.kwonlyargs:
            out.add(a.arg)
        if args.vararg:
            out.add(args.vararg.arg)
        if args.kwarg:
            out.add(args.kwarg.arg)

    def visit(n: ast.AST) -> None:
        if isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
            out.add(n.name)
            for d in getattr(n, "decorator_list", []):
                visit(d)
            return
        if isinstance(n, ast.Lambda):
            return
        if isinstance(n, (ast.Import, ast.ImportFrom)):
            for a in n.names:
                out.add((a.asname or a.name).split(".")[0])
        elif isinstance(n, (ast.Assign,)):
            for t in n.targets:
                out.update(_targets(t))
        elif isinstance(n, (ast.AnnAssign, ast.AugAssign)):
            out.update(_targets(n.target))
        elif isinstance(n, (ast.For, ast.AsyncFor)):
            out.update(_targets(n.target))
        elif isinstance(n, (ast.With, ast.AsyncWith)):
            for it in n.items:
                if it.optional_vars is not None:
                    out.update(_targets(it.optional_vars))
        elif isinstance(n, ast.ExceptHandler) and n.name:
            out.add(n.name)
        elif isinstance(n, ast.NamedExpr):
            out.update(_targets(n.target))
        elif isinstance(n, (ast.Global, ast.Nonlocal)):
            out.update(n.names)
        if isinstance(n, (ast.ListComp, ast.SetComp, ast.DictComp, ast.GeneratorExp)):
            # comprehension scopes are checked on their own; walrus leaks out
            for sub in ast.walk(n):
                if isinstance(sub, ast.NamedExpr):
                    out.update(_targets(sub.target))
            return
        for c in ast.iter_child_nodes(n):
            visit(c)

    for s in body:
        visit(s)
    return out


class Checker:
    def __init__(self, path: Path, tree: ast.Module):
        self.path = path
        self.tree = tree
        self.findings: List[Tuple[int, str]] = []

    def run(self) -> None:
        g = _bound_in(self.tree.body) | BUILTINS
        self._scope(self.tree.body, [g], None)

    def _scope(self, body, stack: List[Set[str]], args) -> None:
        for s in body:
            self._stmt(s, stack)

    def _stmt(self, n: ast.AST, stack: List[Set[str]]) -> None:
        if isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef)):
            for d in n.decorator_list:
                self._expr(d, stack)
            self._args_defaults(n.args, stack)
            inner = _bound_in(n.body, n.args)
            # class bodies are not visible to their methods
            outer = [s for s in stack if not getattr(s, "_class", False)]
            for s in n.body:
                self._stmt(s, outer + [inner])
            return
        if isinstance(n, ast.ClassDef):
            for b in n.bases + [k.value for k in n.keywords] + n.decorator_list:
                self._expr(b, stack)
            cls = _ClassScope(_bound_in(n.body))
            for s in n.body:
                self._stmt(s, stack + [cls])
            return
        for c in ast.iter_child_nodes(n):
            if isinstance(c, ast.stmt):
                self._stmt(c, stack)
            else:
                self._expr(c, stack)

    def _args_defaults(self, a: ast.arguments, stack) -> None:
        for d in a.defaults + [x for x in a.kw_defaults if x is not None]:
            self._expr(d, stack)

    def _expr(self, n: ast.AST, stack: List[Set[str]]) -> None:
        if isinstance(n, ast.Name):
            if isinstance(n.ctx, ast.Load) and not any(n.id in s for s in stack):
                self.findings.append((n.lineno, n.id))
            return
        if isinstance(n, ast.Lambda):
            self._args_defaults(n.args, stack)
            self._expr(n.body, stack + [_bound_in([], n.args)])
            return
        if isinstance(n, (ast.ListComp, ast.SetComp, ast.DictComp, ast.GeneratorExp)):
            local: Set[str] = set()
            st = stack + [local]
            for i, g in enumerate(n.generators):
                # the first iterable is evaluated in the enclosing scope
                self._expr(g.iter, stack if i == 0 else st)
                local.update(_targets(g.target))
                for cond in g.ifs:
                    self._expr(cond, st)
            for sub in ast.walk(n):
                if isinstance(sub, ast.NamedExpr):
                    local.update(_targets(sub.target))
            if isinstance(n, ast.DictComp):
                self._expr(n.key, st)
                self._expr(n.value, st)
            else:
                self._expr(n.elt, st)
            return
        for c in ast.iter_child_nodes(n):
            if isinstance(c, ast.stmt):
                self._stmt(c, stack)
            else:
                self._expr(c, stack)


class _ClassScope(set):
    _class = True


def check(paths: Iterable[Path]) -> List[str]:
    out = []
    for p in paths:
        src = p.read_text()
        try:
            tree = ast.parse(src, str(p))
        except SyntaxError as e:
            out.append(f"{p}:{e.lineno}: syntax error {e.msg}")
            continue
        c = Checker(p, tree)
        c.run()
        out += [f"{p}:{ln}: undefined name {nm!r}" for ln, nm in c.findings]
    return out


def main(argv: List[str]) -> int:
    roots = [Path(a) for a in argv] or [Path(__file__).resolve().parent.parent / "llm_message_queue_amd"]
    files = []
    for r in roots:
        files += sorted(r.rglob("*.py")) if r.is_dir() else [r]
    found = check(files)
    for f in found:
        print(f)
    return 1 if found else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
