"""YAML config with ``--key=value`` overrides — same contract as the reference
``speakerlab/utils/config.py:7-52`` (``Config`` exposes top-level keys as attributes)."""
import os

import yaml


class Config(object):
    def __init__(self, conf_dict):
        self.__dict__.update(conf_dict)


def convert_to_yaml(overrides):
    """['--a=1', '--b', '2'] -> 'a: 1\\nb: 2' (reference config.py:13-27)."""
    tokens = '='.join(overrides).split('=')
    lines = []
    for tok in tokens:
        if tok.startswith('--'):
            lines.append(tok[2:] + ':')
        elif lines:
            lines[-1] += ' ' + tok
    return '\n'.join(lines)


def yaml_config_loader(conf_file, overrides=None):
    with open(conf_file) as f:
        conf = yaml.load(f, Loader=yaml.SafeLoader)
    if overrides is not None:
        conf.update(yaml.load(overrides, Loader=yaml.SafeLoader) or {})
    return conf


def build_config(config_file, overrides=None, copy=False):
    if not config_file.endswith('.yaml'):
        raise ValueError('Unknown config file format')
    conf = yaml_config_loader(config_file, convert_to_yaml(overrides) if overrides is not None else None)
    if copy and 'exp_dir' in conf:
        os.makedirs(conf['exp_dir'], exist_ok=True)
        with open(os.path.join(conf['exp_dir'], 'config.yaml'), 'w') as f:
            f.write(yaml.dump(conf))
    return Config(conf)
