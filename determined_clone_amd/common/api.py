"""HTTP session to the master's REST API (reference: `harness/determined/common/api/_session.py`,
`request.py`). JSON in, JSON out; bearer-token auth; bounded retries on connection errors."""
import json
import logging
import time
from typing import Any, Dict, Optional

import requests

from determined_clone_amd import errors

logger = logging.getLogger("determined_clone_amd.api")


class Session:
    def __init__(self, master_url: str, token: Optional[str] = None, max_retries: int = 5,
                 timeout: float = 60.0) -> None:
        if not master_url.startswith("http"):
            master_url = "http://" + master_url
        self.master = master_url.rstrip("/")
        self.token = token
        self.max_retries = max_retries
        self.timeout = timeout
        self._http = requests.Session()

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
                                       timeout=timeout or self.timeout)
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
