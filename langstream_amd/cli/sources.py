"""Application, instance and secrets paths given to the CLI: local, ``file://``,
``https://`` and GitHub repositories.

Parity: ``langstream-cli/.../commands/BaseCmd.java:430-487`` (``checkFileExistsOrDownload``
/ ``downloadHttpsFile``) and ``commands/applications/GithubRepositoryDownloader.java``:

* ``http://`` is refused ("http is not supported. Please use https instead.");
* ``https://github.com/<owner>/<repo>/tree|blob/<branch>[/<directory>]`` clones the
  repository (``git`` over ``https://github.com/<owner>/<repo>.git``) into the local
  repository cache ``<cli home>/ghrepos/<owner>/<repo>/<branch>``, which later calls
  update instead of re-cloning (``--disable-local-repositories-cache``: a fresh temporary
  clone), and one process clones a repository once even when the app, the instance and
  the secrets all come from it; the result is ``<clone>/<directory>``;
* any other ``https://`` URL is downloaded to a temporary file (HTTP status >= 400
  fails with the status and body);
* ``file://<path>`` is the local path; a local path that does not exist fails.

``LANGSTREAM_GITHUB_URL`` replaces ``https://github.com`` as the clone base (an internal
mirror, or a local directory of bare repositories in tests).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import tempfile
import time
import urllib.parse
from typing import Callable, Dict, Optional, Tuple

_cloned: Dict[Tuple[str, str, str], str] = {}


def cli_home() -> str:
    """The CLI's home directory (where the config file lives: ``~/.langstream``)."""
    return os.path.dirname(os.path.expanduser(os.environ.get("LANGSTREAM_CLI_CONFIG", "~/.langstream/config.yaml")))


def log(msg: str) -> None:
    print(msg, flush=True)


def parse_github(url: str) -> Tuple[str, str, str, str]:
    """``GithubRepositoryDownloader.parseRequest``: (owner, repository, branch, directory)."""
    path = urllib.parse.urlparse(url).path
    parts = path.split("/", 5)
    if len(parts) < 5:
        raise ValueError("Invalid github url. Expected format: "
                         "https://github.com/<owner>/<repository>/tree|blob/<branch>[/directory]")
    return parts[1], parts[2], parts[4], parts[5] if len(parts) > 5 else ""


def _git(args, cwd: Optional[str] = None) -> str:
    r = subprocess.run(["git", *args], cwd=cwd, capture_output=True, text=True,
                       env=dict(os.environ, GIT_TERMINAL_PROMPT="0"))
    if r.returncode != 0:
        raise IOError(f"git {' '.join(args)} failed: {r.stderr.strip() or r.stdout.strip()}")
    return r.stdout.strip()


def _clone(owner: str, repo: str, branch: str, dest: str) -> None:
    base = os.environ.get("LANGSTREAM_GITHUB_URL", "https://github.com").rstrip("/")
    start = time.time()
    log(f"Cloning GitHub repository {owner}/{repo} locally")
    _git(["clone", "--depth", "1", "--branch", branch, f"{base}/{owner}/{repo}.git", dest])
    log(f"Downloaded GitHub repository ({int(time.time() - start)} s)")


def _update(dest: str, branch: str) -> str:
    _git(["fetch", "--depth", "1", "origin", branch], cwd=dest)
    _git(["reset", "--hard", "FETCH_HEAD"], cwd=dest)
    return _git(["rev-parse", "HEAD"], cwd=dest)


def download_github(url: str, use_cache: bool = True) -> str:
    owner, repo, branch, directory = parse_github(url)
    ref = (owner, repo, branch)
    dest = _cloned.get(ref) if use_cache else None
    if dest is not None:
        log(f"Using cached GitHub repository {dest}")
    else:
        home = cli_home()
        if use_cache and home:
            dest = os.path.join(home, "ghrepos", owner, repo, branch)
            try:
                if os.path.isdir(os.path.join(dest, ".git")):
                    log(f"Updating local GitHub repository {dest}")
                    sha = _update(dest, branch)
                    log(f"Updated local GitHub repository to {sha}")
                else:
                    os.makedirs(os.path.dirname(dest), exist_ok=True)
                    shutil.rmtree(dest, ignore_errors=True)
                    _clone(owner, repo, branch, dest)
            except IOError:
                log(f"Failed to update local GitHub repository {url}, falling back to cloning to a "
                    f"temporary directory")
                shutil.rmtree(os.path.join(home, "ghrepos"), ignore_errors=True)
                dest = tempfile.mkdtemp(prefix="langstream")
                shutil.rmtree(dest)
                _clone(owner, repo, branch, dest)
        else:
            dest = tempfile.mkdtemp(prefix="langstream")
            shutil.rmtree(dest)
            _clone(owner, repo, branch, dest)
        _cloned[ref] = dest
    return os.path.join(dest, directory) if directory else dest


def download_https(url: str, fetch: Optional[Callable[[str], Tuple[int, bytes]]] = None) -> str:
    start = time.time()
    if fetch is None:
        import requests
        r = requests.get(url, timeout=120)
        status, body = r.status_code, r.content
    else:
        status, body = fetch(url)
    if status >= 400:
        raise RuntimeError(f"Failed to download file: {url}\nReceived status code: {status}\n"
                           f"{body.decode(errors='replace')}")
    fd, path = tempfile.mkstemp(prefix="langstream", suffix=".bin")
    with os.fdopen(fd, "wb") as f:
        f.write(body)
    log(f"downloaded remote file {url} ({int(time.time() - start)} s)")
    return path


def check_file_exists_or_download(path: Optional[str], use_cache: bool = True) -> Optional[str]:
    if path is None:
        return None
    if path.startswith("http://"):
        raise ValueError("http is not supported. Please use https instead.")
    if path.startswith("https://"):
        if urllib.parse.urlparse(path).hostname == "github.com":
            return download_github(path, use_cache)
        return download_https(path)
    if path.startswith("file://"):
        path = path[len("file://"):]
    if not os.path.exists(path):
        raise FileNotFoundError(f"File {path} does not exist")
    return path


def as_app_directory(path: str) -> str:
    """A downloaded application archive (zip) unpacked to a directory; a directory as is."""
    if os.path.isdir(path):
        return path
    import zipfile
    if not zipfile.is_zipfile(path):
        raise ValueError(f"{path} is neither an application directory nor a zip archive")
    dest = tempfile.mkdtemp(prefix="langstream-app-")
    with zipfile.ZipFile(path) as z:
        for n in z.namelist():
            p = os.path.normpath(os.path.join(dest, n))
            if not p.startswith(os.path.abspath(dest)):
                raise ValueError(f"bad path in archive: {n}")
        z.extractall(dest)
    entries = [e for e in os.listdir(dest) if not e.startswith(".")]
    if not any(e.endswith(".yaml") for e in entries) and len(entries) == 1 and \
            os.path.isdir(os.path.join(dest, entries[0])):
        return os.path.join(dest, entries[0])
    return dest


def _sha512_hex(path: str) -> str:
    import hashlib
    h = hashlib.sha512()
    with open(path, "rb") as f:
        for block in iter(lambda: f.read(1 << 20), b""):
            h.update(block)
    return h.hexdigest()


def _checksum_ok(path: str, sha512sum: Optional[str], logger: Callable[[str], None]) -> bool:
    got = _sha512_hex(path)
    if got != sha512sum:
        logger(f"Computed checksum: {got}")
        logger(f"Expected checksum: {sha512sum}")
    return got == sha512sum


def download_dependencies(directory: str, logger: Callable[[str], None] = log,
                          fetch: Optional[Callable[[str], Tuple[int, bytes]]] = None) -> None:
    """``configuration.dependencies`` of an application directory (``BaseCmd.downloadDependencies``,
    BaseCmd.java:502-582): each ``java-library`` goes to ``java/lib/<file name of the url>``;
    a present file with the right SHA-512 is kept, a corrupted one is replaced, and a
    download that still does not match is deleted and fails the command.  An unreachable
    host only logs: no agent of this runtime loads a java library."""
    import yaml
    conf = os.path.join(directory, "configuration.yaml")
    if not os.path.exists(conf):
        return
    with open(conf, encoding="utf-8") as f:
        data = yaml.safe_load(f) or {}
    deps = (data.get("configuration") or {}).get("dependencies")
    for dep in deps or []:
        url, kind, sha = dep.get("url"), dep.get("type"), dep.get("sha512sum")
        if kind is None:
            raise RuntimeError("dependency type must be set")
        if kind != "java-library":
            raise RuntimeError(f"unsupported dependency type: {kind}")
        out = os.path.join(directory, "java", "lib")
        os.makedirs(out, exist_ok=True)
        target = os.path.join(out, urllib.parse.urlparse(url).path.rsplit("/", 1)[-1])
        if os.path.isfile(target):
            if _checksum_ok(target, sha, logger):
                logger(f"Dependency: {target} at {os.path.abspath(target)}")
                continue
            logger("File seems corrupted, deleting it")
            os.remove(target)
        logger(f"downloading dependency: {target} to {os.path.abspath(target)}")
        try:
            if fetch is None:
                import requests
                r = requests.get(url, timeout=300)
                status, body = r.status_code, r.content
            else:
                status, body = fetch(url)
        except (OSError, IOError) as e:
            # this runtime has no JVM, so no agent loads a java-library: an unreachable
            # repository (offline hosts) leaves the jar out instead of failing the command
            logger(f"dependency not downloaded ({e}); java libraries are not loaded by this runtime")
            continue
        if status >= 400:
            raise IOError(f"Failed to download dependency {url}: HTTP {status}")
        with open(target, "wb") as f:
            f.write(body)
        if not _checksum_ok(target, sha, logger):
            logger("File still seems corrupted. Please double check the checksum and try again.")
            os.remove(target)
            raise IOError(f"File at {url}, seems corrupted")
        logger("dependency downloaded")
