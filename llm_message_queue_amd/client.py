"""Python client for the gateway's REST API.

The reference documents an SDK shape (`docs/api.md:834-887`:
``LLMQueueClient.send_message / get_message / get_queue_status /
health_check`` over ``requests``) but ships none.  This client covers every
route of ``api/server.py``, sends the configured credentials (API key header
or JWT bearer), unwraps the optional ``{"code","message","data"}`` envelope,
and raises ``APIError`` (with the HTTP status, the server's message, the
documented business ``error_code`` and ``Retry-After``) on errors.

    from llm_message_queue_amd.client import LLMQueueClient
    c = LLMQueueClient("http://localhost:8080", api_key="key1")
    mid = c.send_message("conv_1", "user_1", "Hello", priority="high")["message_id"]
    c.wait_for_status(mid, "completed")

``session`` may be any requests-compatible object (``requests.Session``, or
FastAPI's ``TestClient`` in tests).
"""
from __future__ import annotations

import time
from typing import Any, Dict, List, Optional, Union

Priority = Union[int, str, None]


class APIError(Exception):
    def __init__(self, status: int, message: str, error_code: Optional[int] = None,
                 retry_after: Optional[float] = None):
        self.status, self.message, self.error_code, self.retry_after = status, message, error_code, retry_after
        super().__init__(f"HTTP {status}: {message}" + (f" (code {error_code})" if error_code else ""))


class LLMQueueClient:
    def __init__(self, base_url: str = "http://localhost:8080", *, api_key: str = "", api_key_header: str = "X-API-Key",
                 token: str = "", timeout: float = 10.0, session=None, retries_on_429: int = 0):
        self.base = base_url.rstrip("/")
        if self.base.endswith("/api/v1"):
            self.base = self.base[: -len("/api/v1")]
        if session is None:
            import requests
            session = requests.Session()
        self.s = session
        self.timeout = timeout
        self.retries_on_429 = retries_on_429
        self.headers: Dict[str, str] = {"Content-Type": "application/json"}
        if api_key:
            self.headers[api_key_header] = api_key
        if token:
            self.headers["Authorization"] = f"Bearer {token}"

    # ------------------------------------------------------------ transport
    def _call(self, method: str, path: str, body: Any = None, params: Optional[Dict[str, Any]] = None) -> Any:
        url = self.base + path
        kw: Dict[str, Any] = {"headers": self.headers}
        if params:
            kw["params"] = {k: v for k, v in params.items() if v not in (None, "")}
        if body is not None:
            kw["json"] = body
        if self.timeout and not _is_testclient(self.s):
            kw["timeout"] = self.timeout
        attempt = 0
        while True:
            r = self.s.request(method, url, **kw)
            if r.status_code == 429 and attempt < self.retries_on_429:
                attempt += 1
                time.sleep(float(r.headers.get("retry-after", "1") or 1))
                continue
            break
        ctype = r.headers.get("content-type", "")
        data = r.json() if "json" in ctype and r.content else r.text
        if isinstance(data, dict) and "code" in data and ("data" in data or "error" in data) and "timestamp" in data:
            if r.status_code >= 400:                          # envelope error
                raise APIError(r.status_code, data.get("error") or data.get("message", ""), data.get("error_code"),
                               _retry_after(r))
            data = data.get("data")                           # envelope success
        if r.status_code >= 400:
            msg = data.get("error", "") if isinstance(data, dict) else str(data)
            raise APIError(r.status_code, msg, None, _retry_after(r))
        return data

    # ------------------------------------------------------------ health / metrics
    def health_check(self) -> Dict[str, Any]:
        return self._call("GET", "/health")

    def metrics_text(self) -> str:
        return self._call("GET", "/metrics")

    def metrics(self) -> Dict[str, Any]:
        return self._call("GET", "/api/v1/metrics")

    # ------------------------------------------------------------ messages
    def send_message(self, conversation_id: str, user_id: str, content: str, priority: Priority = None,
                     metadata: Optional[Dict[str, Any]] = None, **extra) -> Dict[str, Any]:
        body: Dict[str, Any] = {"conversation_id": conversation_id, "user_id": user_id, "content": content}
        if priority not in (None, ""):
            body["priority"] = priority
        if metadata:
            body["metadata"] = metadata
        body.update(extra)
        return self._call("POST", "/api/v1/messages", body)

    def get_message(self, message_id: str) -> Dict[str, Any]:
        return self._call("GET", f"/api/v1/messages/{message_id}")

    def list_messages(self, user_id: str = "", conversation_id: str = "", status: str = "", limit: int = 10,
                      offset: int = 0) -> Dict[str, Any]:
        return self._call("GET", "/api/v1/messages", params={"user_id": user_id, "conversation_id": conversation_id,
                                                             "status": status, "limit": limit, "offset": offset})

    def update_message_status(self, message_id: str, status: str) -> Dict[str, Any]:
        return self._call("PUT", f"/api/v1/messages/{message_id}/status", {"status": status})

    def delete_message(self, message_id: str) -> Dict[str, Any]:
        return self._call("DELETE", f"/api/v1/messages/{message_id}")

    def wait_for_status(self, message_id: str, status: str = "completed", timeout: float = 30.0,
                        poll: float = 0.02) -> Dict[str, Any]:
        t0 = time.monotonic()
        while True:
            m = self.get_message(message_id)
            if m.get("status") == status:
                return m
            if time.monotonic() - t0 > timeout:
                raise TimeoutError(f"message {message_id} still {m.get('status')!r} after {timeout} s")
            time.sleep(poll)

    # ------------------------------------------------------------ conversations
    def create_conversation(self, user_id: str, metadata: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
        return self._call("POST", "/api/v1/conversations", {"user_id": user_id, "metadata": metadata or {}})

    def get_conversation(self, conversation_id: str) -> Dict[str, Any]:
        return self._call("GET", f"/api/v1/conversations/{conversation_id}")

    def list_conversations(self, user_id: str = "", state: str = "", limit: int = 20, offset: int = 0):
        return self._call("GET", "/api/v1/conversations", params={"user_id": user_id, "state": state,
                                                                  "limit": limit, "offset": offset})

    def update_conversation(self, conversation_id: str, **fields) -> Dict[str, Any]:
        return self._call("PUT", f"/api/v1/conversations/{conversation_id}", fields)

    def add_conversation_message(self, conversation_id: str, user_id: str, content: str,
                                 priority: Priority = None, **extra) -> Dict[str, Any]:
        body: Dict[str, Any] = {"user_id": user_id, "content": content}
        if priority not in (None, ""):
            body["priority"] = priority
        body.update(extra)
        return self._call("POST", f"/api/v1/conversations/{conversation_id}/messages", body)

    def update_conversation_state(self, conversation_id: str, state: str,
                                  metadata: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
        body: Dict[str, Any] = {"state": state}
        if metadata:
            body["metadata"] = metadata
        return self._call("PUT", f"/api/v1/conversations/{conversation_id}/state", body)

    def user_conversations(self, user_id: str) -> List[Dict[str, Any]]:
        return self._call("GET", f"/api/v1/users/{user_id}/conversations")["conversations"]

    # ------------------------------------------------------------ queues / resources / endpoints
    def get_queue_stats(self) -> Dict[str, Any]:
        return self._call("GET", "/api/v1/queues/stats")

    def get_queue_status(self) -> Dict[str, Any]:
        return self._call("GET", "/api/v1/queues/status")

    def register_resource(self, resource: Dict[str, Any]) -> Dict[str, Any]:
        return self._call("POST", "/api/v1/resources", resource)

    def list_resources(self) -> List[Dict[str, Any]]:
        return self._call("GET", "/api/v1/resources")["resources"]

    def resource_stats(self) -> Dict[str, Any]:
        return self._call("GET", "/api/v1/resources/stats")

    def register_endpoint(self, endpoint: Dict[str, Any]) -> Dict[str, Any]:
        return self._call("POST", "/api/v1/endpoints", endpoint)

    def remove_endpoint(self, endpoint_id: str) -> Dict[str, Any]:
        return self._call("DELETE", f"/api/v1/endpoints/{endpoint_id}")

    def set_endpoint_status(self, endpoint_id: str, status: str) -> Dict[str, Any]:
        return self._call("PUT", f"/api/v1/endpoints/{endpoint_id}/status", {"status": status})

    def list_endpoints(self) -> List[Dict[str, Any]]:
        return self._call("GET", "/api/v1/endpoints")["endpoints"]

    def endpoint_stats(self) -> Dict[str, Any]:
        return self._call("GET", "/api/v1/endpoints/stats")

    # ------------------------------------------------------------ admin
    def add_priority_rule(self, priority: Priority, pattern: str) -> Dict[str, Any]:
        return self._call("POST", "/api/v1/admin/preprocessor/rules", {"priority": priority, "pattern": pattern})

    def list_priority_rules(self) -> List[Dict[str, Any]]:
        return self._call("GET", "/api/v1/admin/preprocessor/rules")["rules"]

    def remove_priority_rule(self, priority: Priority, pattern: str) -> Dict[str, Any]:
        return self._call("DELETE", "/api/v1/admin/preprocessor/rules", {"priority": priority, "pattern": pattern})

    def set_user_priority(self, user_id: str, priority: Priority) -> Dict[str, Any]:
        return self._call("POST", "/api/v1/admin/preprocessor/user-priorities",
                          {"user_id": user_id, "priority": priority})

    def remove_queued_message(self, queue_type: str, message_id: str) -> Dict[str, Any]:
        return self._call("DELETE", f"/api/v1/admin/queues/{queue_type}/{message_id}")

    def dead_letters(self) -> List[Dict[str, Any]]:
        return self._call("GET", "/api/v1/admin/dead-letter")["items"]

    def requeue_dead_letter(self, message_id: str) -> Dict[str, Any]:
        return self._call("POST", f"/api/v1/admin/dead-letter/requeue/{message_id}")

    def requeue_all_dead_letters(self) -> Dict[str, Any]:
        return self._call("POST", "/api/v1/admin/dead-letter/requeue-all")

    def get_config(self) -> Dict[str, Any]:
        return self._call("GET", "/api/v1/config")


def _retry_after(r) -> Optional[float]:
    v = r.headers.get("retry-after")
    try:
        return float(v) if v is not None else None
    except ValueError:
        return None


def _is_testclient(s) -> bool:
    return type(s).__name__ == "TestClient"
