"""``det.import_from_path``: import modules from a directory (e.g. an old checkpoint's
``model_def.py``) next to same-named modules already imported, and forget them afterwards
(reference: `harness/determined/_import.py`)."""
import contextlib
import os
import sys
from typing import Dict, Iterator

_active = False


def _under(mod: object, root: str) -> bool:
    f = getattr(mod, "__file__", None)
    return bool(f) and os.path.abspath(f).startswith(root + os.sep)


@contextlib.contextmanager
def import_from_path(path: "os.PathLike[str] | str") -> Iterator[None]:
    """Inside the block, ``import x`` resolves against ``path`` first (shadowing modules of the
    current directory that were already imported); on exit the modules loaded from ``path`` are
    dropped and the previous ``sys.path`` / ``sys.modules`` entries restored. Not reentrant."""
    global _active
    if _active:
        raise RuntimeError("import_from_path does not support nesting or concurrent use")
    root = os.path.abspath(os.fspath(path))
    cwd = os.path.abspath(os.getcwd())
    saved_path = list(sys.path)
    # modules imported from the working directory would satisfy `import x` before `root` does
    shadowed: Dict[str, object] = {k: m for k, m in list(sys.modules.items())
                                   if _under(m, cwd) and not _under(m, root)}
    for k in shadowed:
        del sys.modules[k]
    sys.path = [root] + [p for p in sys.path if p not in ("", cwd)]
    dont_write = sys.dont_write_bytecode
    sys.dont_write_bytecode = True  # leave no __pycache__ in a checkpoint directory
    _active = True
    try:
        yield
    finally:
        _active = False
        sys.dont_write_bytecode = dont_write
        for k in [k for k, m in list(sys.modules.items()) if _under(m, root)]:
            del sys.modules[k]
        sys.path = saved_path
        sys.modules.update(shadowed)  # type: ignore[arg-type]
