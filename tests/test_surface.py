"""CPU: the reference's public surface on the hot path resolves through the
drop-in.  tests/golden/reference_surface.json (tests/golden/make_surface.py:
the reference's in-scope modules read with `ast`) lists every public class,
method and function with its positional parameters; in a fresh interpreter
whose sys.path is ofdm-lte_amd/compat only, each must import under the
reference's module name with the same positional parameters (a mirror may
add keyword-only arguments, e.g. precision=).  The reference modules'
self-test functions (test_layer_mapper, test_mimo_detector,
test_rank_adaptation: demo printouts) are not part of the surface."""
import json
import os
import subprocess
import sys

from conftest import ROOT

SURFACE = os.path.join(ROOT, 'tests', 'golden', 'reference_surface.json')

CHECK = r'''
import importlib, inspect, json, sys
spec = json.load(open(sys.argv[1]))['modules']
bad = []
def pos(obj, method):
    try:
        sig = inspect.signature(obj)
    except (TypeError, ValueError):
        return None
    ps = [p for p in sig.parameters.values()
          if p.kind in (p.POSITIONAL_ONLY, p.POSITIONAL_OR_KEYWORD)]
    names = [p.name for p in ps]
    return names
def cmp(where, obj, want, method):
    got = pos(obj, method)
    if got is None:
        bad.append(f'{where}: no signature')
    elif got != want['positional']:
        bad.append(f'{where}: positional {got} != reference {want["positional"]}')
n = 0
for mod, s in spec.items():
    try:
        m = importlib.import_module(mod)
    except Exception as e:
        bad.append(f'{mod}: import failed: {type(e).__name__}: {e}')
        continue
    for name in s.get('reexports', []):
        n += 1
        if not hasattr(m, name):
            bad.append(f'{mod}.{name}: missing (re-export)')
    for fn, want in s['functions'].items():
        if fn.startswith('test_'):
            continue
        n += 1
        f = getattr(m, fn, None)
        if f is None:
            bad.append(f'{mod}.{fn}: missing')
            continue
        cmp(f'{mod}.{fn}', f, want, False)
    for cls, meths in s['classes'].items():
        n += 1
        c = getattr(m, cls, None)
        if c is None:
            bad.append(f'{mod}.{cls}: missing')
            continue
        for meth, want in meths.items():
            n += 1
            a = inspect.getattr_static(c, meth, None)
            if a is None:
                bad.append(f'{mod}.{cls}.{meth}: missing')
                continue
            if want.get('property'):
                if not isinstance(a, property):
                    bad.append(f'{mod}.{cls}.{meth}: not a property')
                continue
            f = a.__func__ if isinstance(a, (staticmethod, classmethod)) else a
            want2 = dict(want)
            if not isinstance(a, staticmethod):   # unbound: drop self
                got = pos(f, True)
                if got is not None:
                    got = got[1:]
                if got != want['positional']:
                    bad.append(f'{mod}.{cls}.{meth}: positional {got} != reference {want["positional"]}')
            else:
                cmp(f'{mod}.{cls}.{meth}', f, want, False)
print(json.dumps({'checked': n, 'bad': bad}))
'''


def run_check():
    env = dict(os.environ)
    env['PYTHONPATH'] = os.path.join(ROOT, 'ofdm-lte_amd', 'compat')
    r = subprocess.run([sys.executable, '-c', CHECK, SURFACE], env=env, capture_output=True, text=True, timeout=300,
                       cwd='/tmp')
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_reference_surface_resolves_with_same_positional_args():
    out = run_check()
    assert out['checked'] > 250
    assert not out['bad'], '\n'.join(out['bad'])
