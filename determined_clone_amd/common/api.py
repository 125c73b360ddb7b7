"""HTTP session to the master's REST API (reference: `harness/determined/common/api/_session.py`,
`request.py`). JSON in, JSON out; bearer-token auth; bounded retries on connection errors."""
import json
import logging
import os
import time
from typing import Any, Dict, Optional

import requests
import requests.adapters

from determined_clone_amd import errors

logger = logging.getLogger("determined_clone_amd.api")


class Cert:
    """How to verify an HTTPS master (reference: `harness/determined/common/api/certs.py`).

    ``bundle``: a CA / self-signed certificate file to trust, or ``False`` for no verification
    (``DET_MASTER_CERT_FILE=noverify``), or ``None`` for the system store. ``name``: the host name
    the certificate was issued for, when it differs from the address dialed
    (``DET_MASTER_CERT_NAME``)."""

    def __init__(self, bundle: Any = None, name: Optional[str] = None, noverify: bool = False) -> None:
        self.bundle = False if noverify else bundle
        self.name = name

    @classmethod
    def from_env(cls) -> "Cert":
        f = os.environ.get("DET_MASTER_CERT_FILE")
        name = os.environ.get("DET_MASTER_CERT_NAME") or None
        if f and f.lower() == "noverify":
            return cls(noverify=True, name=name)
        return cls(bundle=f or None, name=name)


class _NamedHostAdapter(requests.adapters.HTTPAdapter):
    """Checks the master's certificate against ``cert_name`` instead of the dialed host."""

    def __init__(self, cert_name: str, **kw: Any) -> None:
        self._cert_name = cert_name
        super().__init__(**kw)

    def init_poolmanager(self, *args: Any, **kw: Any) -> None:
        kw["assert_hostname"] = self._cert_name
        kw["server_hostname"] = self._cert_name
        super().init_poolmanager(*args, **kw)


class Session:
    def __init__(self, master_url: str, token: Optional[str] = None, max_retries: int = 5,
                 timeout: float = 60.0, cert: Optional[Cert] = None) -> None:
        if not master_url.startswith("http"):
            master_url = "http://" + master_url
        self.master = master_url.rstrip("/")
        self.token = token
        self.max_retries = max_retries
        self.timeout = timeout
        self.cert = cert if cert is not None else Cert.from_env()
        self._http = requests.Session()
        # per-request ``verify`` (requests lets REQUESTS_CA_BUNDLE override a session-level one)
        self._verify: Any = True
        if self.master.startswith("https://"):
            if self.cert.bundle is not None:
                self._verify = self.cert.bundle
            if self.cert.name:
                self._http.mount("https://", _NamedHostAdapter(self.cert.name))

    def _headers(self) -> Dict[str, str]:
        h = {"Content-Type": "application/json"}
        if self.token:
            h["Authorization"] = f"Bearer {self.token}"
        return h

    def request(self, method: str, path: str, body: Any = None, params: Optional[Dict] = None,
                timeout: Optional[float] = None, raw: bool = False) -> Any:
        url = self.master + path
        data = None if body is None else json.dumps(body, default=_default)
        last: Optional[BaseException] = None
        for attempt in range(self.max_retries + 1):
            try:
                r = self._http.request(method, url, data=data, params=params, headers=self._headers(),
                                       timeout=timeout or self.timeout, verify=self._verify)
            except requests.ConnectionError as e:
                last = e
                time.sleep(min(2 ** attempt * 0.2, 5.0))
                continue
            if r.status_code == 404:
                raise errors.NotFoundException(_msg(r))
            if r.status_code == 401:
                raise errors.UnauthenticatedException(_msg(r))
            if r.status_code == 403:
                raise errors.ForbiddenException(_msg(r))
            if r.status_code >= 400:
                raise errors.APIException(r.status_code, _msg(r))
            if raw:
                return r.content
            if not r.content:
                return None
            return r.json()
        raise errors.MasterNotFoundException(f"could not reach master at {self.master}: {last}")

    def get(self, path: str, params: Optional[Dict] = None, **kw: Any) -> Any:
        return self.request("GET", path, params=params, **kw)

    def post(self, path: str, body: Any = None, **kw: Any) -> Any:
        return self.request("POST", path, body=body if body is not None else {}, **kw)

    def patch(self, path: str, body: Any = None, **kw: Any) -> Any:
        return self.request("PATCH", path, body=body if body is not None else {}, **kw)

    def put(self, path: str, body: Any = None, **kw: Any) -> Any:
        return self.request("PUT", path, body=body if body is not None else {}, **kw)

    def delete(self, path: str, **kw: Any) -> Any:
        return self.request("DELETE", path, **kw)


def _msg(r: requests.Response) -> str:
    try:
        j = r.json()
        return j.get("error") or j.get("message") or r.text
    except ValueError:
        return r.text


def _default(o: Any) -> Any:
    from determined_clone_amd.util import to_python

    v = to_python(o)
    return str(v) if v is o else v
