"""Browser UI served by the master (reference: the React app under `webui/react/src`, pages in
`webui/react/src/pages/*.tsx` -- Dashboard, ExperimentList/Details, TrialDetails, Cluster,
JobQueue, TaskList/TaskLogs, InteractiveTask, ModelRegistry/ModelDetails/ModelVersionDetails,
WorkspaceList/Details, ProjectDetails, WebhookList, Admin users, ClusterLogs, SignIn).

The reference builds a React bundle with npm; this image has no JS toolchain, so the UI is one
dependency-free single-page app (``static/app.js``, hash routes, SVG metric charts) that talks to
the same ``/api/v1`` REST surface as the CLI and SDK. The master serves it at ``/det/`` (and
redirects ``/`` there); the session token lives in ``localStorage`` and is passed to task
services (notebooks, TensorBoards, shells) through the ``/proxy/{task}/?token=`` hand-off."""
import mimetypes
import os
from typing import Optional, Tuple

STATIC_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "static")
_TYPES = {".js": "text/javascript; charset=utf-8", ".css": "text/css; charset=utf-8",
          ".html": "text/html; charset=utf-8", ".svg": "image/svg+xml"}


def resolve(path: str) -> Optional[Tuple[str, bytes]]:
    """Map a request path under ``/det`` to ``(content_type, body)``; every path that is not a
    static asset is the SPA shell (``index.html``). ``None`` for paths outside ``/det``."""
    if path in ("/det", "/det/"):
        rel = "index.html"
    elif path.startswith("/det/static/"):
        rel = path[len("/det/static/"):]
    elif path.startswith("/det/"):
        rel = "index.html"
    else:
        return None
    full = os.path.realpath(os.path.join(STATIC_DIR, rel))
    if not full.startswith(STATIC_DIR + os.sep) or not os.path.isfile(full):
        return None
    ext = os.path.splitext(full)[1]
    ctype = _TYPES.get(ext) or mimetypes.guess_type(full)[0] or "application/octet-stream"
    with open(full, "rb") as f:
        return ctype, f.read()
