#!/usr/bin/env python3
"""Golden vectors for the tile hierarchy (reference py/get_tiles.py:30-171).

TEST INFRASTRUCTURE ONLY.  Runs ONCE in the build container, where the reference
checkout exists.  It loads the reference's own classes BoundingBox / TileHierarchy /
Tiles (get_tiles.py:22-102) and its listing loop (the body of the main block after
check_args, :134-171) from the source text by AST extraction, and executes them under
Python 2 semantics: `long` is int, `/` between ints floors (Tiles.Digits' `number /=
10`), and the TileHierarchy.levels dict iterates its keys as Python 2 does (keys 0, 1,
2: small ints sit in hash slots 0, 1, 2).  Only the resulting input/output data are
written (tests/golden/tile_cases.json); tests never read the reference.

Usage:  python tests/golden/make_tile_goldens.py [--ref /root/reference]
"""
import argparse
import ast
import io
import json
import math
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def py2_div(a, b):
    if isinstance(a, int) and isinstance(b, int):
        return a // b
    return a / b


class _Py2(ast.NodeTransformer):
    """`/` -> _py2_div, `x /= y` -> x = _py2_div(x, y)."""

    def visit_BinOp(self, node):
        self.generic_visit(node)
        if isinstance(node.op, ast.Div):
            return ast.copy_location(ast.Call(func=ast.Name(id='_py2_div', ctx=ast.Load()),
                                              args=[node.left, node.right], keywords=[]), node)
        return node

    def visit_AugAssign(self, node):
        self.generic_visit(node)
        if isinstance(node.op, ast.Div) and isinstance(node.target, ast.Name):
            call = ast.Call(func=ast.Name(id='_py2_div', ctx=ast.Load()),
                            args=[ast.Name(id=node.target.id, ctx=ast.Load()), node.value], keywords=[])
            return ast.copy_location(ast.Assign(targets=[ast.Name(id=node.target.id, ctx=ast.Store())],
                                                value=call), node)
        return node


class Py2Dict(dict):
    """A dict iterated in Python 2's order for small non-negative int keys."""

    def items(self):
        return sorted(dict.items(self))


def load(ref):
    path = os.path.join(ref, 'py', 'get_tiles.py')
    tree = ast.parse(open(path).read(), filename=path)
    keep = [n for n in tree.body if isinstance(n, (ast.ClassDef, ast.Assign))]
    main = next(n for n in tree.body if isinstance(n, ast.If))  # if __name__ == "__main__":
    # the listing loop: every statement after check_args(...) and TileHierarchy()
    body = [s for s in main.body if not (isinstance(s, ast.Expr) and isinstance(s.value, ast.Call) and
                                         getattr(s.value.func, 'id', '') == 'check_args')]
    fn = ast.FunctionDef(name='_listing', args=ast.arguments(posonlyargs=[], args=[], vararg=None, kwonlyargs=[],
                                                             kw_defaults=[], kwarg=None, defaults=[]),
                         body=[ast.Global(names=['boundingbox', 'suffix'])] + body, decorator_list=[])
    mod = ast.Module(body=keep + [fn], type_ignores=[])
    mod = ast.fix_missing_locations(_Py2().visit(mod))
    env = {'math': math, 'long': int, '_py2_div': py2_div, '__name__': 'get_tiles_golden'}
    exec(compile(mod, path, 'exec'), env)
    # TileHierarchy.levels iterated in Python 2 order
    orig_init = env['TileHierarchy'].__init__

    def init(self):
        orig_init(self)
        self.levels = Py2Dict(self.levels)
    env['TileHierarchy'].__init__ = init
    return env


def listing(env, bbox, suffix):
    env['boundingbox'] = bbox
    env['suffix'] = suffix
    buf, old = io.StringIO(), sys.stdout
    sys.stdout = buf
    try:
        env['_listing']()
    finally:
        sys.stdout = old
    return buf.getvalue().splitlines()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--ref', default='/root/reference')
    a = ap.parse_args()
    env = load(a.ref)
    rng = random.Random(8032)
    th = env['TileHierarchy']()
    cases = {'row': [], 'col': [], 'file': [], 'listing': []}
    ys = [-90, 90, -90.0001, 90.0001, 0, 0.25, -0.25, 40.512764, -33.9, 89.99, 45.0, 44.999999]
    xs = [-180, 180, -180.0001, 180.0001, 0, 1, -1, -74.251961, 151.2, 179.99, -0.125, 120.0]
    ys += [rng.uniform(-91, 91) for _ in range(40)]
    xs += [rng.uniform(-181, 181) for _ in range(40)]
    for lv in (0, 1, 2):
        t = th.levels[lv]
        cases['row'] += [{'level': lv, 'y': y, 'row': t.Row(y)} for y in ys]
        cases['col'] += [{'level': lv, 'x': x, 'col': t.Col(x)} for x in xs]
        ids = [0, 1, 999, 1000, t.max_tile_id, t.max_tile_id - 1] + [rng.randrange(t.max_tile_id) for _ in range(30)]
        env['suffix'] = 'gph'
        cases['file'] += [{'level': lv, 'tile_id': i, 'suffix': 'gph', 'file': t.GetFile(i, lv)} for i in ids]
    boxes = ['-74.251961,40.512764,-73.755405,40.903125', '-0.5,51.2,0.3,51.7', '179.5,-17.2,-179.7,-16.4',
             '-180,-1,-179,1', '170,10,190,11', '-190,10,-170,11', '13.0,52.3,13.8,52.7', '0,0,0,0', '-1,-1,1,1']
    for _ in range(6):
        x0, y0 = rng.uniform(-179, 178), rng.uniform(-80, 79)
        boxes.append('%.6f,%.6f,%.6f,%.6f' % (x0, y0, x0 + rng.uniform(0.01, 1.2), y0 + rng.uniform(0.01, 1.2)))
    for b in boxes:
        for suf in ('gph', 'json'):
            cases['listing'].append({'bbox': b, 'suffix': suf, 'files': listing(env, b, suf)})
    with open(os.path.join(HERE, 'tile_cases.json'), 'w') as f:
        json.dump({'generator': 'tests/golden/make_tile_goldens.py',
                   'source': 'reference py/get_tiles.py classes and listing loop executed under py2 semantics',
                   'cases': cases}, f, separators=(',', ':'))
    print({k: len(v) for k, v in cases.items()}, sum(len(c['files']) for c in cases['listing']), 'files')


if __name__ == '__main__':
    main()
