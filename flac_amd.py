"""Import shim: the package lives in ``flac-py_amd/`` (a directory name Python cannot
import directly), so this module makes it importable as ``flac_amd``.

``import flac_amd.encoder`` resolves submodules from ``flac-py_amd/``.
"""
import os as _os

__path__ = [_os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "flac-py_amd")]
with open(_os.path.join(__path__[0], "__init__.py")) as _f:
    exec(compile(_f.read(), _os.path.join(__path__[0], "__init__.py"), "exec"))

if __name__ == "__main__":  # python -m flac_amd encode in.wav out.flac ...
    import sys as _sys

    from flac_amd.cli import main as _main
    _sys.exit(_main())
