"""HTTP error carried from a handler to the server (the role tornado.web.HTTPError
plays in python/kfserving/kfserving/handlers/http.py:35-50 and kfserver.py:127-196)."""
from http import HTTPStatus


class HTTPError(Exception):
    def __init__(self, status_code: int = 500, reason: str = None):
        self.status_code = int(status_code)
        self.reason = reason or HTTPStatus(self.status_code).phrase
        super().__init__(f"HTTP {self.status_code}: {self.reason}")
