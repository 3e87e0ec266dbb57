"""The website the config-4 bench's webcrawler-source walks (bench.py): /step/<n>/
index.html lists that step's pages and links the next step's index, which long-polls
until the bench publishes the step.

It is the crawl TARGET, not part of the pipeline under test, so by default rank 0 runs
it in its own process (``SiteProcess``): serving a step's pages (256 at 8 GPUs) from
rank 0's interpreter took GIL time from that rank's agents and engine.  ``publish`` /
``close`` go over the child's stdin.
"""
from __future__ import annotations

import argparse
import sys
import threading


def make_page(i: int, corpus) -> str:
    """A crawled page: ~12 paragraphs of corpus sentences."""
    return "\n\n".join(" ".join(corpus[(i * 31 + p * 7 + j) % len(corpus)] for j in range(5)) for p in range(12))


class Site:
    """Local HTTP site the crawler walks: /step/<n>/index.html lists that step's pages
    and links the next step's index, which long-polls until the step is published."""

    def __init__(self, corpus, per_step: int):
        import http.server
        self.corpus, self.per_step = corpus, per_step
        self.published = -1
        self.cv = threading.Condition()
        site = self

        class H(http.server.BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"
            # headers and body leave in separate writes: with Nagle on, the body waits for
            # the client's delayed ACK of the headers (~40 ms per page on loopback)
            disable_nagle_algorithm = True

            def log_message(self, *a):
                pass

            def do_GET(self):
                parts = self.path.strip("/").split("/")
                if len(parts) != 3 or parts[0] != "step":
                    return self._send(404, b"")
                step = int(parts[1])
                with site.cv:
                    site.cv.wait_for(lambda: site.published >= step, timeout=1800)
                if site.published < step:
                    return self._send(503, b"")
                if parts[2] == "index.html":
                    links = "".join(f'<a href="/step/{step}/{d}.html">p{d}</a>' for d in range(site.per_step))
                    body = f'<html><body>{links}<a href="/step/{step + 1}/index.html">next</a></body></html>'
                else:
                    d = int(parts[2].split(".")[0])
                    text = make_page(step * site.per_step + d, site.corpus)
                    body = "<html><body>" + "".join(f"<p>{p}</p>" for p in text.split("\n\n")) + "</body></html>"
                self._send(200, body.encode())

            def _send(self, code, body):
                try:
                    self.send_response(code)
                    self.send_header("Content-Type", "text/html; charset=utf-8")
                    self.send_header("Content-Length", str(len(body)))
                    self.end_headers()
                    self.wfile.write(body)
                except (BrokenPipeError, ConnectionResetError):
                    # the crawler gave up on a long-polled index (its http-timeout, or the
                    # bench ending): nothing to answer, and no traceback on stderr
                    self.close_connection = True

        self.httpd = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.httpd.daemon_threads = True
        self.url = f"http://127.0.0.1:{self.httpd.server_address[1]}"
        threading.Thread(target=self.httpd.serve_forever, daemon=True).start()

    def publish(self, step: int) -> None:
        with self.cv:
            self.published = step
            self.cv.notify_all()

    def close(self) -> None:
        self.publish(1 << 30)
        self.httpd.shutdown()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--per-step", type=int, required=True)
    ap.add_argument("--corpus-sentences", type=int, required=True)
    a = ap.parse_args(argv)
    from ..tokenizers import builtin_corpus
    site = Site(builtin_corpus(a.corpus_sentences), a.per_step)
    print(f"url={site.url}", flush=True)
    for line in sys.stdin:
        cmd = line.split()
        if cmd and cmd[0] == "publish":
            site.publish(int(cmd[1]))
    site.close()
    return 0


class SiteProcess:
    """``Site`` in a child interpreter (started before the parent touches the GPU)."""

    def __init__(self, per_step: int, corpus_sentences: int):
        from ..utils.procs import read_tagged, spawn_module
        self.proc = spawn_module("langstream_amd.bench.site",
                                 ["--per-step", str(per_step), "--corpus-sentences", str(corpus_sentences)])
        self.url = read_tagged(self.proc, "url=", "bench site process")

    def publish(self, step: int) -> None:
        self.proc.stdin.write(f"publish {step}\n")
        self.proc.stdin.flush()

    def close(self) -> None:
        from ..utils.procs import close_stdin_and_wait
        close_stdin_and_wait(self.proc)


if __name__ == "__main__":
    raise SystemExit(main())
