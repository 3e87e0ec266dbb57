"""webcrawler-source.

Parity: ``WebCrawlerSource.java:95-461``, ``crawler/WebCrawler.java``,
``crawler/WebCrawlerConfiguration.java``, ``crawler/WebCrawlerStatus.java:30-238``.

* configuration: ``seed-urls``, ``allowed-domains`` (URL prefix or bare host),
  ``forbidden-paths`` (path prefixes), ``max-urls`` (1000), ``max-depth`` (50),
  ``handle-robots-file`` (true), ``scan-html-documents`` (true), ``user-agent``,
  ``min-time-between-requests`` (500 ms), ``max-error-count`` (5), ``http-timeout``
  (10000 ms), ``allow-non-html-contents`` (false), ``handle-cookies`` (true),
  ``reindex-interval-seconds`` (86400), ``max-unflushed-pages`` (100),
  ``state-storage`` (``s3`` | ``disk``) with ``bucketName``/``endpoint``/keys for S3.
* crawl order: robots.txt of each seed's host first (crawl-delay, disallow rules,
  sitemaps), then pages breadth-first; links come from ``<a href>`` only; URL
  fragments are stripped; 3xx redirects are followed by enqueueing the Location (unless
  it is forbidden); 4xx drops the URL, 5xx/IO errors re-queue it up to
  ``max-error-count`` times.
* each page is ONE record: key = url, value = the page re-serialised from its parsed
  tree (``agents/htmlnorm.py``, the reference's ``document.html()``) for ``text/*``
  pages, the raw bytes for XML and -- with ``allow-non-html-contents`` -- other types;
  headers ``url`` and ``content_type``.  ``commit()`` marks the URL processed (it leaves ``remainingUrls``);
  status (remaining urls, every seen url with type/depth, robots files, index
  timestamps) is flushed every ``max-unflushed-pages`` commits and at the end of a pass,
  so a restarted agent resumes where it stopped.  After a full pass the source idles
  until ``reindex-interval-seconds`` elapsed, then restarts from the seeds.
"""
from __future__ import annotations

import json
import logging
import os
import re
import threading
import time
import urllib.parse
import urllib.robotparser
from collections import deque
from typing import Any, Callable, Deque, Dict, List, Optional, Set

from ..api.agent import AgentSource
from ..api.record import Header, Record, SimpleRecord
from ..api.util import get_boolean, get_int, get_list, get_string
from ..runtime.registry import register_agent
from . import htmlnorm

log = logging.getLogger(__name__)
DEFAULT_USER_AGENT = "Mozilla/5.0 (compatible; LangStream.ai/0.1; +https://langstream.ai)"
PAGE, ROBOTS, SITEMAP = "PAGE", "ROBOTS", "SITEMAP"
_XML_TYPE = re.compile(r"(application|text)/\w*\+?xml")


def remove_fragment(url: str) -> str:
    i = url.find("#")
    return url if i < 0 else url[:i]


def domain_of(url: str) -> str:
    b = url.find("://")
    if b <= 0:
        return ""
    e = url.find("/", b + 3)
    return url[b + 3:] if e <= 0 else url[b + 3: e]


class CrawlerConfig:
    def __init__(self, allowed_domains: Set[str], forbidden_paths: Set[str], max_urls=1000, max_depth=50,
                 handle_robots=True, scan_html=True, allow_non_html=False, user_agent=DEFAULT_USER_AGENT,
                 min_time_between_requests=500, max_error_count=5, http_timeout=10000, handle_cookies=True):
        self.allowed_domains, self.forbidden_paths = allowed_domains, forbidden_paths
        self.max_urls, self.max_depth = max_urls, max_depth
        self.handle_robots, self.scan_html, self.allow_non_html = handle_robots, scan_html, allow_non_html
        self.user_agent = user_agent
        self.min_time = min_time_between_requests
        self.max_error_count, self.http_timeout, self.handle_cookies = max_error_count, http_timeout, handle_cookies

    def is_allowed_url(self, url: str) -> bool:
        try:
            u = urllib.parse.urlparse(url)
        except ValueError:
            return False
        if not u.scheme or not u.netloc:
            return False
        path = u.path or "/"
        host = u.hostname or ""
        allowed = any(url.startswith(d) or d.lower() == host.lower() for d in self.allowed_domains)
        forbidden = any(path.startswith(p) for p in self.forbidden_paths)
        return allowed and not forbidden


class CrawlerStatus:
    def __init__(self):
        self.last_index_end = 0
        self.last_index_start = 0
        self.remaining: Deque[str] = deque()   # discovered, not committed
        self.pending: Deque[str] = deque()     # discovered, not yet returned by read()
        self.urls: Dict[str, tuple] = {}       # url -> (type, depth)
        self.robots: Dict[str, dict] = {}
        self.errors: Dict[str, int] = {}

    def add_url(self, url: str, typ: str, depth: int, to_scan: bool) -> None:
        url = remove_fragment(url)
        was = url in self.urls
        self.urls[url] = (typ, depth)
        if to_scan and not was:
            self.pending.append(url)
            self.remaining.append(url)

    def next_url(self) -> Optional[str]:
        return self.pending.popleft() if self.pending else None

    def url_processed(self, url: str) -> None:
        try:
            self.remaining.remove(url)
        except ValueError:
            pass
        self.errors.pop(remove_fragment(url), None)

    def temporary_error(self, url: str) -> int:
        url = remove_fragment(url)
        self.urls.pop(url, None)
        n = self.errors.get(url, 0) + 1
        self.errors[url] = n
        return n

    def to_json(self) -> dict:
        return {"remainingUrls": list(self.remaining),
                "urls": [{"url": u, "type": t, "depth": d} for u, (t, d) in self.urls.items()],
                "lastIndexEndTimestamp": self.last_index_end, "lastIndexStartTimestamp": self.last_index_start,
                "robotFiles": self.robots}

    def reload(self, st: Optional[dict]) -> None:
        if not st:
            return
        rem = st.get("remainingUrls") or []
        self.pending = deque(rem)
        self.remaining = deque(rem)
        self.urls = {u["url"]: (u["type"], int(u["depth"])) for u in st.get("urls") or []}
        self.last_index_end = int(st.get("lastIndexEndTimestamp") or 0)
        self.last_index_start = int(st.get("lastIndexStartTimestamp") or 0)
        self.robots = dict(st.get("robotFiles") or {})


class WebCrawler:
    def __init__(self, cfg: CrawlerConfig, status: CrawlerStatus, visitor: Callable[[str, bytes, str], None]):
        import requests
        self.cfg, self.status, self.visitor = cfg, status, visitor
        self.http = requests.Session()
        self.http.headers["User-Agent"] = cfg.user_agent
        if not cfg.handle_cookies:
            from http.cookiejar import DefaultCookiePolicy
            self.http.cookies.set_policy(DefaultCookiePolicy(allowed_domains=[]))
        self.rules: Dict[str, urllib.robotparser.RobotFileParser] = {}
        for url, rf in self.status.robots.items():
            self._apply_robots(url, rf.get("content", ""))

    def crawl(self, start: str) -> None:
        if self._forbidden(start):
            return
        if self.cfg.handle_robots:
            u = urllib.parse.urlparse(start)
            self.status.add_url(f"{u.scheme}://{u.netloc}/robots.txt", ROBOTS, 0, True)
        self._add_page(start, None)

    def restart(self, seeds) -> None:
        self.status.pending.clear()
        self.status.remaining.clear()
        self.status.urls.clear()
        self.status.last_index_start = int(time.time() * 1000)
        for s in seeds:
            self.crawl(s)

    def _add_page(self, url: str, parent_depth: Optional[int]) -> bool:
        depth = 0 if parent_depth is None else parent_depth + 1
        if self.cfg.max_urls > 0 and len(self.status.urls) >= self.cfg.max_urls:
            return False
        if self.cfg.max_depth > 0 and depth > self.cfg.max_depth:
            return False
        self.status.add_url(url, PAGE, depth, True)
        return True

    def _forbidden(self, url: str) -> bool:
        if not self.cfg.is_allowed_url(url):
            return True
        rp = self.rules.get(domain_of(url))
        return rp is not None and not rp.can_fetch(self.cfg.user_agent, url)

    def _throttle(self, url: str) -> None:
        delay = 0.0
        rp = self.rules.get(domain_of(url))
        if rp is not None:
            d = rp.crawl_delay(self.cfg.user_agent)
            delay = float(d) * 1000 if d else 0.0
        if self.cfg.min_time > 0:
            delay = min(self.cfg.min_time, delay) if delay > 0 else self.cfg.min_time
        if delay > 0:
            time.sleep(delay / 1000.0)

    def _temporary_error(self, url: str, typ: str, depth: int) -> None:
        if self.status.temporary_error(url) >= self.cfg.max_error_count:
            self.status.add_url(url, typ, depth, False)
        else:
            self.status.add_url(url, typ, depth, True)

    def _apply_robots(self, url: str, content: str) -> None:
        rp = urllib.robotparser.RobotFileParser()
        rp.parse(content.splitlines())
        self.rules[domain_of(url)] = rp
        return rp

    def run_cycle(self) -> bool:
        cur = self.status.next_url()
        if cur is None:
            return False
        typ, depth = self.status.urls.get(cur, (PAGE, 0))
        timeout = self.cfg.http_timeout / 1000.0
        if typ in (ROBOTS, SITEMAP):
            try:
                r = self.http.get(cur, timeout=timeout)
                body = r.text if r.status_code < 400 else ""
            except Exception:  # noqa: BLE001
                body = ""
            if typ == ROBOTS:
                rp = self._apply_robots(cur, body)
                self.status.robots[cur] = {"content": body, "contentType": "text/plain"}
                for sm in rp.site_maps() or []:
                    self.status.add_url(sm, SITEMAP, 0, True)
            else:
                for loc in re.findall(r"<loc>\s*([^<\s]+)\s*</loc>", body):
                    if not self._forbidden(loc):
                        self._add_page(loc, depth)
            self.status.url_processed(cur)
            return True
        try:
            r = self.http.get(cur, timeout=timeout, allow_redirects=False)
        except Exception as e:  # noqa: BLE001
            log.info("error fetching %s: %s", cur, e)
            self._temporary_error(cur, typ, depth)
            self._throttle(cur)
            return True
        code = r.status_code
        if 300 <= code < 400:
            loc = r.headers.get("Location")
            if loc:
                loc = urllib.parse.urljoin(cur, loc)
                if loc != cur and not self._forbidden(loc):
                    self._add_page(loc, depth)
            self._throttle(cur)
            return True
        if code >= 400:
            if code >= 500:
                self._temporary_error(cur, typ, depth)
            self._throttle(cur)
            return True
        ctype = r.headers.get("Content-Type", "text/html")
        low = ctype.lower()
        # what the reference's HTML fetch accepts (text/*, XML types); XML is passed through
        is_xml = bool(_XML_TYPE.match(low))
        is_html = low.startswith("text/") and not is_xml
        if is_xml:
            self.visitor(cur, r.content, ctype)
            self._throttle(cur)
            return True
        if not is_html:
            if self.cfg.allow_non_html:
                self.visitor(cur, r.content, ctype)
            else:
                self.status.add_url(cur, typ, depth, False)
            self._throttle(cur)
            return True
        try:
            page, hrefs = htmlnorm.normalize(r.text)
            content = page.encode("utf-8")
        except Exception:  # noqa: BLE001
            content, hrefs = r.content, []
        if self.cfg.scan_html:
            for href in hrefs:
                u = remove_fragment(urllib.parse.urljoin(cur, href))
                if not u.startswith(("http://", "https://")):
                    continue
                if self._forbidden(u):
                    self.status.add_url(u, PAGE, depth + 1, False)
                else:
                    self._add_page(u, depth)
        self.visitor(cur, content, ctype)
        self._throttle(cur)
        return True


class _DiskState:
    def __init__(self, path: str):
        self.path = path

    def load(self) -> Optional[dict]:
        try:
            with open(self.path) as f:
                return json.load(f)
        except (OSError, ValueError):
            return None

    def store(self, st: dict) -> None:
        tmp = self.path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(st, f)
        os.replace(tmp, self.path)


class _S3State:
    def __init__(self, client, bucket: str, name: str):
        self.client, self.bucket, self.name = client, bucket, name

    def load(self) -> Optional[dict]:
        b = self.client.get_object(self.bucket, self.name)
        return json.loads(b) if b else None

    def store(self, st: dict) -> None:
        self.client.put_object(self.bucket, self.name, json.dumps(st).encode())


@register_agent("webcrawler-source")
class WebCrawlerSource(AgentSource):
    def init(self, configuration: Dict[str, Any]) -> None:
        self.cfg_raw = dict(configuration)
        self.seeds = list(dict.fromkeys(get_list("seed-urls", configuration)))
        self.reindex_s = get_int("reindex-interval-seconds", 86400, configuration)
        self.max_unflushed = get_int("max-unflushed-pages", 100, configuration)
        self.flush_next = self.max_unflushed
        self.cc = CrawlerConfig(
            set(get_list("allowed-domains", configuration)), set(get_list("forbidden-paths", configuration)),
            get_int("max-urls", 1000, configuration), get_int("max-depth", 50, configuration),
            get_boolean("handle-robots-file", True, configuration),
            get_boolean("scan-html-documents", True, configuration),
            get_boolean("allow-non-html-contents", False, configuration),
            get_string("user-agent", DEFAULT_USER_AGENT, configuration),
            get_int("min-time-between-requests", 500, configuration), get_int("max-error-count", 5, configuration),
            get_int("http-timeout", 10000, configuration), get_boolean("handle-cookies", True, configuration))
        self.status = CrawlerStatus()
        self.status.last_index_start = int(time.time() * 1000)
        self.found: Deque[tuple] = deque()
        self.finished = False
        self.on_reindex_start: Optional[Callable[[], None]] = None
        self._lock = threading.Lock()

    def set_context(self, context) -> None:
        super().set_context(context)
        name = f"{context.global_agent_id}.webcrawler.status.json"
        if get_string("state-storage", "s3", self.cfg_raw) == "disk":
            d = context.get_persistent_state_directory_for_agent(self.agent_id())
            if d is None:
                raise ValueError(f"No local disk path available for agent {self.agent_id()} and state-storage "
                                 f"was set to 'disk'")
            self.state = _DiskState(os.path.join(d, name))
        else:
            from .storage import S3Client
            c = self.cfg_raw
            client = S3Client(get_string("endpoint", "http://minio-endpoint.-not-set:9090", c),
                              get_string("access-key", "minioadmin", c), get_string("secret-key", "minioadmin", c),
                              get_string("region", "", c))
            bucket = get_string("bucketName", "langstream-source", c)
            if not client.bucket_exists(bucket):
                client.make_bucket(bucket)
            self.state = _S3State(client, bucket, name)
        self.status_file = name

    def start(self) -> None:
        self.status.reload(self.state.load())
        self.crawler = WebCrawler(self.cc, self.status, lambda u, b, ct: self.found.append((u, b, ct)))
        for s in self.seeds:
            self.crawler.crawl(s)

    def _flush(self) -> None:
        try:
            self.state.store(self.status.to_json())
        except Exception as e:  # noqa: BLE001
            log.error("cannot persist crawler status: %s", e)

    def read(self) -> List[Record]:
        with self._lock:
            if self.finished:
                self._check_reindex()
                time.sleep(0.1)
                return []
            if not self.found:
                did = self.crawler.run_cycle()
                if not did:
                    self.finished = True
                    self.status.last_index_end = int(time.time() * 1000)
                    self._flush()
                elif not self.found:
                    return []
            if not self.found:
                time.sleep(0.1)
                return []
            url, body, ctype = self.found.popleft()
        self.processed(0, 1)
        return [SimpleRecord(url, body, None, int(time.time() * 1000),
                             [Header("url", url), Header("content_type", ctype)])]

    def _check_reindex(self) -> None:
        if self.reindex_s <= 0 or self.status.last_index_end <= 0:
            return
        if (time.time() * 1000 - self.status.last_index_end) / 1000 >= self.reindex_s:
            if self.on_reindex_start is not None:
                self.on_reindex_start()
            self.crawler.restart(self.seeds)
            self.finished = False
            self._flush()

    def commit(self, records: List[Record]) -> None:
        with self._lock:
            for r in records:
                self.status.url_processed(r.key())
                self.flush_next -= 1
                if self.flush_next <= 0:
                    self._flush()
                    self.flush_next = self.max_unflushed

    def build_additional_info(self) -> Dict[str, Any]:
        return {"seed-Urls": self.seeds, "allowed-domains": sorted(self.cc.allowed_domains),
                "statusFileName": getattr(self, "status_file", None)}
