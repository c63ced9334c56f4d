"""The reference's public Python surface on the hot path, as data: for every
in-scope module of Darioxavierl/OFDM-LTE (SURVEY §8 rows a and f), the
public functions and classes, each class's public methods, and each
callable's positional parameter names -- read from the source files with
`ast` (text only: nothing is imported or executed).  Output:
tests/golden/reference_surface.json, the fixture
tests/test_surface.py checks the drop-in (ofdm-lte_amd/compat) against.

usage:  python tests/golden/make_surface.py
"""
import ast
import json
import os
import sys

REF = '/root/reference'
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'reference_surface.json')

# module path (import name) -> file under the reference
MODULES = {
    'config': 'config.py',
    'ofdm_module': 'ofdm_module.py',
    'core.ofdm_core': 'core/ofdm_core.py',
    'core.channel': 'core/channel.py',
    'core.rayleighchannel': 'core/rayleighchannel.py',
    'core.modulator': 'core/modulator.py',
    'core.resource_mapper': 'core/resource_mapper.py',
    'core.lte_receiver': 'core/lte_receiver.py',
    'core.demodulator': 'core/demodulator.py',
    'core.dft_precoding': 'core/dft_precoding.py',
    'core.mimo_channel_estimator_periodic': 'core/mimo_channel_estimator_periodic.py',
    'core.sfbc_alamouti': 'core/sfbc_alamouti.py',
    'core.layer_mapper': 'core/layer_mapper.py',
    'core.mimo_detector': 'core/mimo_detector.py',
    'core.codebook_lte': 'core/codebook_lte.py',
    'core.rank_adaptation': 'core/rank_adaptation.py',
    'core.beamforming_precoder': 'core/beamforming_precoder.py',
    'core.csi_feedback': 'core/csi_feedback.py',
    'core.channel_coding': 'core/channel_coding/__init__.py',
    'core.channel_coding.crc': 'core/channel_coding/crc.py',
    'core.channel_coding.segmentation': 'core/channel_coding/segmentation.py',
    'core.channel_coding.turbo_encoder': 'core/channel_coding/turbo_encoder.py',
    'core.channel_coding.turbo_decoder': 'core/channel_coding/turbo_decoder.py',
    'core.channel_coding.rate_matching': 'core/channel_coding/rate_matching.py',
    'utils.image_processing': 'utils/image_processing.py',
}


def params(fn, method):
    a = fn.args
    pos = [x.arg for x in a.posonlyargs + a.args]
    if method and pos and pos[0] in ('self', 'cls'):
        pos = pos[1:]
    return {'positional': pos, 'n_defaults': len(a.defaults), 'vararg': bool(a.vararg), 'kwarg': bool(a.kwarg)}


def surface(path):
    tree = ast.parse(open(path, encoding='utf-8-sig').read())
    out = {'functions': {}, 'classes': {}}
    for node in tree.body:
        if isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef)) and not node.name.startswith('_'):
            out['functions'][node.name] = params(node, False)
        elif isinstance(node, ast.ClassDef) and not node.name.startswith('_'):
            meths = {}
            for b in node.body:
                if isinstance(b, (ast.FunctionDef, ast.AsyncFunctionDef)) and (not b.name.startswith('_')
                                                                               or b.name == '__init__'):
                    static = any(isinstance(d, ast.Name) and d.id == 'staticmethod' for d in b.decorator_list)
                    prop = any(isinstance(d, ast.Name) and d.id == 'property' for d in b.decorator_list)
                    meths[b.name] = dict(params(b, not static), property=prop)
            out['classes'][node.name] = meths
    return out


def main():
    if not os.path.isdir(REF):
        sys.exit('make_surface.py reads the reference at /root/reference (survey container only)')
    res = {m: surface(os.path.join(REF, f)) for m, f in MODULES.items()}
    # names a package __init__ re-exports (from .x import a, b)
    tree = ast.parse(open(os.path.join(REF, 'core/channel_coding/__init__.py'), encoding='utf-8-sig').read())
    names = [a.name for n in tree.body if isinstance(n, ast.ImportFrom) for a in n.names]
    res['core.channel_coding']['reexports'] = names
    json.dump({'generated_by': 'tests/golden/make_surface.py (ast of the reference sources)', 'modules': res},
              open(OUT, 'w'), indent=1, sort_keys=True)
    nc = sum(len(v['classes']) for v in res.values())
    nm = sum(len(c) for v in res.values() for c in v['classes'].values())
    nf = sum(len(v['functions']) for v in res.values())
    print(f'{len(res)} modules, {nc} classes, {nm} methods, {nf} functions -> {OUT}')


if __name__ == '__main__':
    main()
