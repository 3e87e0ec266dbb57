"""The reference's crawler state-machine tests, ported
(``langstream-agents/langstream-agent-webcrawler/src/test/java/ai/langstream/agents/webcrawler/crawler/WebCrawlerTest.java``):
one ``run_cycle`` at a time against a stub site, checking the documents handed to the
visitor, the pending queue and the set of known URLs after every step -- 5xx and
connection resets re-queue a URL until ``max-error-count``, 4xx drop it, redirects
enqueue their target unless it is forbidden, binary content passes through with
``allow-non-html-contents``.  WireMock is ``ref_runtime_harness.FakeHTTP``."""
from __future__ import annotations

import pytest

from ref_runtime_harness import FakeHTTP
from langstream_amd.agents.webcrawler import CrawlerConfig, CrawlerStatus, WebCrawler


@pytest.fixture()
def site():
    w = FakeHTTP()
    yield w
    w.close()


def _crawler(site, **kw):
    cfg = CrawlerConfig({site.url}, set(), handle_robots=False, min_time_between_requests=0, **kw)
    status, docs = CrawlerStatus(), []
    c = WebCrawler(cfg, status, lambda url, content, ctype: docs.append((url, content, ctype)))
    c.crawl(site.url + "/index.html")
    return c, status, docs


def _state(status):
    return len(status.pending), len(status.urls)


def test_web_site_errors(site):
    """WebCrawlerTest.testWebSiteErrors: 503 re-queues, 404 drops, a recovered page is read."""
    site.stub("GET", "/index.html", ctype="text/html",
              text='<a href="internalErrorPage.html">link</a>\n<a href="notFoundPage.html">link</a>\n')
    site.stub("GET", "/internalErrorPage.html", status=503)
    site.stub("GET", "/notFoundPage.html", status=404)
    c, status, docs = _crawler(site, max_error_count=5)
    c.run_cycle()
    assert [d[0] for d in docs] == [site.url + "/index.html"]
    assert _state(status) == (2, 3)
    c.run_cycle()                     # internalErrorPage: 503, back in the queue
    assert _state(status) == (2, 3)
    c.run_cycle()                     # notFoundPage: 404, dropped
    assert _state(status) == (1, 3)
    c.run_cycle()                     # internalErrorPage again
    assert _state(status) == (1, 3)
    site.stub("GET", "/internalErrorPage.html", ctype="text/html", text="ok !\n")
    c.run_cycle()
    assert _state(status) == (0, 3)


def test_web_site_permanent_errors(site):
    """WebCrawlerTest.testWebSitePermanentErrors: after max-error-count (3) the URL is given up."""
    site.stub("GET", "/index.html", ctype="text/html", text='<a href="internalErrorPage.html">link</a>\n')
    site.stub("GET", "/internalErrorPage.html", status=503)
    c, status, docs = _crawler(site, max_error_count=3)
    c.run_cycle()
    assert [d[0] for d in docs] == [site.url + "/index.html"] and _state(status) == (1, 2)
    c.run_cycle()
    assert _state(status) == (1, 2)
    c.run_cycle()
    assert _state(status) == (1, 2)
    c.run_cycle()
    assert _state(status) == (0, 2)
    assert c.run_cycle() is False     # nothing to do


def test_redirects(site):
    """WebCrawlerTest.testRedirects: a redirect enqueues its target (not reported as a
    document itself); a redirect off the allowed domains is dropped."""
    site.stub("GET", "/index.html", ctype="text/html",
              text='<a href="redirectToGoodWebsite.html">link</a>\n<a href="redirectToBadWebsite.html">link</a>\n')
    site.stub("GET", "/redirectToGoodWebsite.html", status=307,
              response_headers={"Location": site.url + "/goodWebsite.html"})
    site.stub("GET", "/redirectToBadWebsite.html", status=307,
              response_headers={"Location": "http://go-away-from-here/somewhere.html"})
    site.stub("GET", "/goodWebsite.html", ctype="text/html", text="ok")
    c, status, docs = _crawler(site)
    c.run_cycle()
    assert [d[0] for d in docs] == [site.url + "/index.html"] and _state(status) == (2, 3)
    c.run_cycle()                     # redirectToGoodWebsite
    assert _state(status) == (2, 4) and len(docs) == 1
    c.run_cycle()                     # redirectToBadWebsite
    assert _state(status) == (1, 4)
    c.run_cycle()                     # goodWebsite
    assert _state(status) == (0, 4)
    assert [d[0] for d in docs] == [site.url + "/index.html", site.url + "/goodWebsite.html"]
    assert c.run_cycle() is False


def test_network_errors(site):
    """WebCrawlerTest.testNetworkErrors: connection resets re-queue the URL; it is read once
    the server answers again."""
    site.stub("GET", "/index.html", ctype="text/html", text='<a href="internalErrorPage.html">link</a>\n')
    site.stub("GET", "/internalErrorPage.html", status=FakeHTTP.RESET)
    c, status, docs = _crawler(site, max_error_count=5)
    c.run_cycle()
    assert [d[0] for d in docs] == [site.url + "/index.html"] and _state(status) == (1, 2)
    c.run_cycle()
    assert _state(status) == (1, 2)
    c.run_cycle()
    assert _state(status) == (1, 2)
    site.stub("GET", "/internalErrorPage.html", ctype="text/html", text="ok !\n")
    c.run_cycle()
    assert _state(status) == (0, 2)


def test_network_errors_eventually_fail(site):
    """WebCrawlerTest.testNetworkErrorsEventuallyFail: max-error-count 1 gives up at once."""
    site.stub("GET", "/index.html", ctype="text/html", text='<a href="internalErrorPage.html">link</a>\n')
    site.stub("GET", "/internalErrorPage.html", status=FakeHTTP.RESET)
    c, status, docs = _crawler(site, max_error_count=1)
    c.run_cycle()
    assert [d[0] for d in docs] == [site.url + "/index.html"] and _state(status) == (1, 2)
    c.run_cycle()
    assert _state(status) == (0, 2)


def test_binary_content(site):
    """WebCrawlerTest.testBinaryContent: a PDF link is fetched and handed over as bytes with
    its content type."""
    pdf = bytes([1, 2, 3, 4, 5])
    site.stub("GET", "/index.html", ctype="text/html", text='<a href="document.pdf">link</a>\n')
    site.stub("GET", "/document.pdf", data=pdf, ctype="application/pdf")
    c, status, docs = _crawler(site, allow_non_html=True, max_error_count=5)
    c.run_cycle()
    assert [d[0] for d in docs] == [site.url + "/index.html"] and _state(status) == (1, 2)
    c.run_cycle()
    assert docs[1] == (site.url + "/document.pdf", pdf, "application/pdf")
    assert _state(status) == (0, 2)
