"""Import alias for the ``hierarchical-vision_amd/`` package directory.

A hyphen cannot appear in a Python import name, so this module makes the
directory importable as ``hvamd``: ``import hvamd.swinv2`` resolves to
``hierarchical-vision_amd/swinv2.py``.
"""
import os as _os

__path__ = [_os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "hierarchical-vision_amd")]
with open(_os.path.join(__path__[0], "__init__.py")) as _f:
    exec(compile(_f.read(), _os.path.join(__path__[0], "__init__.py"), "exec"))
