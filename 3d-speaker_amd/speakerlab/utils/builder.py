"""Object construction from ``{'obj': dotted.path, 'args': {...}}`` specs with ``<name>``
references into a Config — same contract as the reference ``speakerlab/utils/builder.py:9-91``.
Because this package keeps the reference's dotted paths, registry strings such as
``speakerlab.models.eres2net.ERes2NetV2.ERes2NetV2`` resolve to the MI355X modules."""
import importlib
import re

from speakerlab.utils.config import Config

_REF = re.compile(r'^<[a-zA-Z]\w*>$')


def dynamic_import(import_path):
    module, _, name = import_path.rpartition('.')
    return getattr(importlib.import_module(module), name)


def is_ref_type(value: str):
    assert isinstance(value, str), 'Input value is not a str.'
    return bool(_REF.match(value))


def _is_spec(x):
    return isinstance(x, dict) and 'obj' in x and 'args' in x


def is_built(ins):
    if _is_spec(ins):
        return False
    if isinstance(ins, dict):
        return all(is_built(v) for v in ins.values())
    if isinstance(ins, list):
        return all(is_built(v) for v in ins)
    if isinstance(ins, str):
        return is_built(ins.split('/')) if '/' in ins else not is_ref_type(ins)
    return True


def deep_build(ins, config, build_space: set = None):
    if is_built(ins):
        return ins
    build_space = set() if build_space is None else build_space
    if isinstance(ins, list):
        ins[:] = [deep_build(v, config, build_space) for v in ins]
        return ins
    if _is_spec(ins):
        assert isinstance(ins['args'], dict), f"Args for {ins['obj']} must be a dict."
        return dynamic_import(ins['obj'])(**deep_build(ins['args'], config, build_space))
    if isinstance(ins, dict):
        for k in ins:
            ins[k] = deep_build(ins[k], config, build_space)
        return ins
    if isinstance(ins, str):
        if '/' in ins:
            return '/'.join(deep_build(ins.split('/'), config, build_space))
        if is_ref_type(ins):
            ref = ins[1:-1]
            if ref in build_space:
                raise ValueError('Cross referencing is not allowed in config.')
            assert hasattr(config, ref), f'Key name {ins} not found in config.'
            build_space.add(ref)
            val = deep_build(getattr(config, ref), config, build_space)
            setattr(config, ref, val)
            build_space.remove(ref)
            return val
    return ins


def build(name: str, config: Config):
    return deep_build(f'<{name}>', config)
