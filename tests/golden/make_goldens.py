#!/usr/bin/env python3
"""Generate the golden vectors that pin the post-match stages of the hot path.

TEST INFRASTRUCTURE ONLY.  This script runs ONCE, in the build container, where the
reference checkout exists at /root/reference.  It loads three pieces of the
reference's own pure-Python code from the source text at run time (AST extraction,
nothing is copied into this repository):

  * ``report()``                        py/reporter_service.py:79-179
  * the privacy-cull ``while`` loop     py/simple_reporter.py:221-239
  * the report filter + hour bucketing  py/simple_reporter.py:176-196

and executes them under Python-2 arithmetic semantics (the reference is Python 2):
``round`` is half-away-from-zero on the exact binary value and ``int / int`` floors.
Inputs are synthetic meili-style segment lists (schema: README.md:288-300).  The
resulting input/output pairs are written as JSON data under tests/golden/; only
those data files are used by the tests (they never read /root/reference).

Usage:  python tests/golden/make_goldens.py  [--ref /root/reference]
"""
import argparse
import ast
import json
import math
import os
import random
from decimal import Decimal, ROUND_HALF_UP

HERE = os.path.dirname(os.path.abspath(__file__))


def py2_round(x, n=0):
    """Python 2.7 float round(): half away from zero on the exact binary value."""
    if math.isinf(x) or math.isnan(x):
        return x
    q = Decimal(1).scaleb(-n)
    return float(Decimal(x).quantize(q, rounding=ROUND_HALF_UP))


def py2_div(a, b):
    """Python 2 ``/``: floor division for two ints, true division otherwise."""
    if isinstance(a, int) and isinstance(b, int):
        return a // b
    return a / b


class _Py2Div(ast.NodeTransformer):
    def visit_BinOp(self, node):
        self.generic_visit(node)
        if isinstance(node.op, ast.Div):
            return ast.copy_location(
                ast.Call(func=ast.Name(id='_py2_div', ctx=ast.Load()),
                         args=[node.left, node.right], keywords=[]), node)
        return node


def _load(path):
    with open(path) as f:
        return ast.parse(f.read(), filename=path)


def _compile_fn(fn_node, filename, env):
    mod = ast.Module(body=[fn_node], type_ignores=[])
    mod = ast.fix_missing_locations(_Py2Div().visit(mod))
    exec(compile(mod, filename, 'exec'), env)
    return env[fn_node.name]


def extract_report(ref):
    path = os.path.join(ref, 'py', 'reporter_service.py')
    tree = _load(path)
    fn = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == 'report')
    env = {'math': math, 'round': py2_round, '_py2_div': py2_div}
    return _compile_fn(fn, path, env)


def extract_cull(ref):
    """Wrap the reference's cull `while` loop (simple_reporter.py:221-239) in a function."""
    path = os.path.join(ref, 'py', 'simple_reporter.py')
    tree = _load(path)
    rep = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == 'report')
    loop = next(n for n in ast.walk(rep) if isinstance(n, ast.For))
    body = loop.body
    w = next(i for i, n in enumerate(body) if isinstance(n, ast.While))
    # the two initialisers `start = 0`, `i = 0` precede the while loop
    stmts = body[w - 2:w + 1]
    fn = ast.FunctionDef(
        name='cull', args=ast.arguments(posonlyargs=[], args=[ast.arg('segments'), ast.arg('privacy')],
                                        kwonlyargs=[], kw_defaults=[], defaults=[]),
        body=stmts + [ast.Return(value=ast.Name(id='segments', ctx=ast.Load()))],
        decorator_list=[], returns=None, type_comment=None)
    env = {'_py2_div': py2_div}
    return _compile_fn(fn, path, env)


def extract_bucketing(ref):
    """Wrap simple_reporter.py:176-196 (filter + hour bucketing of one trace's reports)."""
    path = os.path.join(ref, 'py', 'simple_reporter.py')
    tree = _load(path)
    consts = {}
    for n in tree.body:  # LEVEL_BITS ... INVALID_SEGMENT_ID, get_tile_level/index (36-49)
        if isinstance(n, ast.Assign) and isinstance(n.targets[0], ast.Name) and \
                n.targets[0].id.isupper():
            exec(compile(ast.fix_missing_locations(ast.Module(body=[n], type_ignores=[])), path, 'exec'), consts)
    helpers = [n for n in tree.body if isinstance(n, ast.FunctionDef)
               and n.name in ('get_tile_level', 'get_tile_index')]
    match = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == 'match')
    # the statements after the Match/report try-block inside the per-window loop
    win_loop = [n for n in ast.walk(match) if isinstance(n, ast.For)
                and isinstance(n.target, ast.Tuple) and n.target.elts[0].id == 'idx'][0]
    t = next(i for i, n in enumerate(win_loop.body) if isinstance(n, ast.Try))
    stmts = win_loop.body[t + 1:]
    args = ['points', 'report', 'quantisation', 'mode', 'source', 'dest_dir', 'tiles', 'uuid', 'file_name']
    fn = ast.FunctionDef(
        name='bucket', args=ast.arguments(posonlyargs=[], args=[ast.arg(a) for a in args],
                                          kwonlyargs=[], kw_defaults=[], defaults=[]),
        body=stmts + [ast.Return(value=ast.Name(id='tiles', ctx=ast.Load()))],
        decorator_list=[], returns=None, type_comment=None)

    class _Log:
        def error(self, *a, **k):
            pass

    env = dict(consts)
    env.update({'math': math, 'round': py2_round, '_py2_div': py2_div, 'os': os,
                'logger': _Log(), 'str': py2_str})
    for h in helpers:
        _compile_fn(h, path, env)
    return _compile_fn(fn, path, env), consts['INVALID_SEGMENT_ID']


def py2_str(x):
    """Python 2 str(): floats print with 12 significant digits (repr-like for ints)."""
    if isinstance(x, float):
        s = '%.12g' % x
        if 'e' not in s and '.' not in s and 'inf' not in s and 'nan' not in s:
            s += '.0'
        return s
    return str(x)


# --------------------------------------------------------------------------------------
# synthetic meili-style segment lists (README.md:288-300)
# --------------------------------------------------------------------------------------
def mk_id(rng, level):
    tile = rng.randrange(0, 1 << 22)
    idx = rng.randrange(0, 1 << 21)
    return (idx << 25) | (tile << 3) | level


def random_segments(rng, n, t0):
    segs = []
    t = float(t0)
    shape = 0
    for k in range(n):
        kind = rng.random()
        seg = {}
        if kind < 0.12:
            seg['internal'] = True
        elif kind < 0.22:
            seg['internal'] = False       # unassociated (no segment_id)
        else:
            seg['segment_id'] = mk_id(rng, rng.choice([0, 0, 1, 1, 2]))
            seg['internal'] = False
        dur = rng.choice([0.0, rng.uniform(0.2, 3), rng.uniform(3, 90), rng.uniform(90, 400)])
        length = rng.choice([rng.randint(1, 30), rng.randint(30, 900), rng.randint(900, 4000)])
        st = t
        et = t + dur
        if k == 0 or rng.random() < 0.1:
            st = -1
        if k == n - 1 or rng.random() < 0.1:
            et = -1
        seg['start_time'] = round(st, 3) if st != -1 else -1
        seg['end_time'] = round(et, 3) if et != -1 else -1
        seg['length'] = length if (st != -1 and et != -1 and 'segment_id' in seg) else -1
        if rng.random() < 0.05 and 'segment_id' in seg:
            seg['length'] = 0
        seg['queue_length'] = rng.choice([0, 0, 0, rng.randint(0, 200)])
        seg['begin_shape_index'] = shape
        shape += rng.randint(0, 4)
        seg['end_shape_index'] = shape
        seg['way_ids'] = [rng.randrange(1, 1 << 31) for _ in range(rng.randint(1, 3))]
        segs.append(seg)
        t = et if et != -1 else t + rng.uniform(1, 30)
        if rng.random() < 0.05:
            t -= rng.uniform(0, 5)         # non-monotonic → invalid_times
    return segs


def report_cases(report, rng):
    cases = []
    hand = []
    A, B, C = mk_id(rng, 0), mk_id(rng, 1), mk_id(rng, 2)
    # complete → complete, transition level; README example shape
    hand.append([{'segment_id': A, 'start_time': 1000.0, 'end_time': 1030.0, 'length': 400,
                  'queue_length': 0, 'internal': False, 'begin_shape_index': 0, 'end_shape_index': 3},
                 {'segment_id': B, 'start_time': 1030.0, 'end_time': 1060.0, 'length': 500,
                  'queue_length': 0, 'internal': False, 'begin_shape_index': 3, 'end_shape_index': 7},
                 {'segment_id': C, 'start_time': 1060.0, 'end_time': -1, 'length': -1,
                  'queue_length': 0, 'internal': False, 'begin_shape_index': 7, 'end_shape_index': 9}])
    # internal between two complete segments keeps the prior
    hand.append([{'segment_id': A, 'start_time': 100.0, 'end_time': 130.5, 'length': 420,
                  'queue_length': 0, 'internal': False, 'begin_shape_index': 0, 'end_shape_index': 2},
                 {'internal': True, 'start_time': 130.5, 'end_time': 133.0, 'length': -1,
                  'queue_length': 0, 'begin_shape_index': 2, 'end_shape_index': 2},
                 {'segment_id': B, 'start_time': 133.0, 'end_time': 170.0, 'length': 333,
                  'queue_length': 0, 'internal': False, 'begin_shape_index': 2, 'end_shape_index': 5},
                 {'segment_id': A, 'start_time': 170.0, 'end_time': 260.0, 'length': 420,
                  'queue_length': 0, 'internal': False, 'begin_shape_index': 5, 'end_shape_index': 9}])
    # too fast (>160 km/h) and dt<=0
    hand.append([{'segment_id': A, 'start_time': 10.0, 'end_time': 12.0, 'length': 900,
                  'queue_length': 0, 'internal': False, 'begin_shape_index': 0, 'end_shape_index': 1},
                 {'segment_id': B, 'start_time': 12.0, 'end_time': 12.0, 'length': 50,
                  'queue_length': 0, 'internal': False, 'begin_shape_index': 1, 'end_shape_index': 2},
                 {'segment_id': A, 'start_time': 12.0, 'end_time': 100.0, 'length': 50,
                  'queue_length': 0, 'internal': False, 'begin_shape_index': 2, 'end_shape_index': 3},
                 {'segment_id': C, 'start_time': 100.0, 'end_time': 300.0, 'length': 50,
                  'queue_length': 0, 'internal': False, 'begin_shape_index': 3, 'end_shape_index': 8}])
    # discontinuity: partial end followed by partial start
    hand.append([{'segment_id': A, 'start_time': 10.0, 'end_time': -1, 'length': -1,
                  'queue_length': 0, 'internal': False, 'begin_shape_index': 0, 'end_shape_index': 4},
                 {'segment_id': B, 'start_time': -1, 'end_time': 80.0, 'length': -1,
                  'queue_length': 0, 'internal': False, 'begin_shape_index': 5, 'end_shape_index': 7},
                 {'segment_id': C, 'start_time': 80.0, 'end_time': 200.0, 'length': 700,
                  'queue_length': 0, 'internal': False, 'begin_shape_index': 7, 'end_shape_index': 12}])
    # empty
    hand.append([])
    for segs in hand:
        end = max([s['end_time'] for s in segs] + [s['start_time'] for s in segs] + [0]) + 20
        cases.append((segs, [{'lat': 0.0, 'lon': 0.0, 'time': int(end)}], 15, [0, 1], [0, 1]))
    for k in range(110):
        segs = random_segments(rng, rng.randint(0, 16), rng.randint(1, 1 << 30))
        last = max([s['end_time'] for s in segs] + [s['start_time'] for s in segs] + [0])
        end = int(last + rng.choice([0, 5, 14, 15, 16, 40, 300]))
        levels = rng.choice([[0, 1], [0, 1, 2], [0], [1, 2], []])
        trans = rng.choice([[0, 1], [0, 1, 2], [0], [2], []])
        thr = rng.choice([15, 15, 0, 5, 30])
        cases.append((segs, [{'lat': 0.0, 'lon': 0.0, 'time': end - 1}, {'lat': 0.0, 'lon': 0.0, 'time': end}],
                      thr, levels, trans))
    out = []
    for segs, trace, thr, lv, tl in cases:
        seg_in = json.loads(json.dumps({'segments': segs}))
        res = report(json.loads(json.dumps(seg_in)), {'trace': trace}, thr, set(lv), set(tl))
        out.append({'segments': seg_in, 'trace': trace, 'threshold_sec': thr,
                    'report_levels': lv, 'transition_levels': tl,
                    'expected': json.loads(json.dumps(res))})
    return out


def cull_cases(cull, rng):
    out = []
    hand = [
        (['A,B,1\n', 'A,B,2\n', 'C,D,1\n'], 2),   # trailing singleton merged into preceding run
        (['A,B,1\n', 'C,D,1\n'], 2),
        (['A,B,1\n'], 2),
        (['A,B,1\n', 'A,B,1\n'], 2),
        ([], 2),
        (['A,B,1\n', 'C,D,1\n', 'C,D,2\n', 'E,F,1\n'], 2),
        (['A,B,1\n', 'A,B,2\n', 'A,B,3\n', 'C,D,1\n', 'C,D,1\n'], 3),
    ]
    for lines, p in hand:
        out.append({'lines': lines, 'privacy': p, 'expected': cull(list(lines), p)})
    for k in range(200):
        n = rng.randint(0, 30)
        pairs = ['%d,%d' % (rng.randint(1, 6), rng.randint(1, 3)) for _ in range(n)]
        lines = sorted('%s,%d,1\n' % (pr, rng.randint(0, 99)) for pr in pairs)
        p = rng.choice([1, 2, 2, 3, 5])
        out.append({'lines': lines, 'privacy': p, 'expected': cull(list(lines), p)})
    return out


def bucket_cases(bucket, rng):
    out = []
    for k in range(120):
        t_first = rng.randint(1483228800, 1483228800 + 86400 * 30)
        span = rng.choice([30, 600, 3599, 3600, 7200, 20000])
        t_last = t_first + rng.randint(1, span)
        reports = []
        for _ in range(rng.randint(0, 16)):
            t0 = rng.choice([rng.uniform(t_first - 10, t_last), -1.0, 0.0, float(t_first)])
            t1 = t0 + rng.choice([rng.uniform(0, 0.5), rng.uniform(0.5, 2000), 0.5, 1.5, 2.5, -3.0, 9000.0])
            r = {'id': mk_id(rng, rng.choice([0, 1, 2])), 't0': round(t0, 3), 't1': round(t1, 3),
                 'length': rng.choice([rng.randint(1, 3000)] * 4 + [0, -1]),
                 'queue_length': rng.choice([0, 0, 0, 0, 17, -1])}
            if rng.random() < 0.7:
                r['next_id'] = mk_id(rng, rng.choice([0, 1, 2]))
            reports.append(r)
        q = rng.choice([3600, 3600, 900])
        mode = rng.choice(['auto', 'bicycle'])
        points = [{'time': t_first}, {'time': t_last}]
        tiles = bucket(points, {'datastore': {'reports': reports}}, q, mode, 'smpl_rprt', 'D', {}, 'u', 'f')
        out.append({'first_time': t_first, 'last_time': t_last, 'reports': reports, 'quantisation': q,
                    'mode': mode, 'source': 'smpl_rprt',
                    'expected': {k2: v for k2, v in sorted(tiles.items())}})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--ref', default='/root/reference')
    a = ap.parse_args()
    rng = random.Random(20171)
    report = extract_report(a.ref)
    cull = extract_cull(a.ref)
    bucket, invalid = extract_bucketing(a.ref)
    assert invalid == 0x3fffffffffff
    data = {
        'report_cases.json': report_cases(report, rng),
        'cull_cases.json': cull_cases(cull, rng),
        'bucket_cases.json': bucket_cases(bucket, rng),
    }
    for name, d in data.items():
        with open(os.path.join(HERE, name), 'w') as f:
            json.dump({'generator': 'tests/golden/make_goldens.py',
                       'source': 'reference pure-Python functions executed under py2 semantics',
                       'cases': d}, f, separators=(',', ':'))
        print(name, len(d), 'cases')


if __name__ == '__main__':
    main()
