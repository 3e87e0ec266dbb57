"""agents/htmlnorm.py: the crawler's page re-serialisation.  The three pages of the
reference's WebCrawlerSourceIT pin the layout exactly (tests/test_ref_runtime_io.py); the
cases here pin this module's tree building and escaping rules (parity beyond those pages
is unpinned: no jsoup offline)."""
from langstream_amd.agents.htmlnorm import normalize, parse


def test_reference_pages():
    assert normalize('<a href="secondPage.html">link</a>\n')[0] == \
        '<html>\n <head></head>\n <body>\n  <a href="secondPage.html">link</a>\n </body>\n</html>'
    assert normalize('  <a href="thirdPage.html">link</a>\n  <a href="index.html">link to home</a>\n')[0] == \
        '<html>\n <head></head>\n <body>\n  <a href="thirdPage.html">link</a> <a href="index.html">link to home' \
        '</a>\n </body>\n</html>'
    assert normalize("  Hello!\n")[0] == "<html>\n <head></head>\n <body>\n  Hello!\n </body>\n</html>"


def test_links_in_document_order_and_only_anchors():
    _, hrefs = normalize('<link href="style.css"><p><a href="a">1</a><img src="x"><a href="b#f">2</a></p>'
                         '<a name="no-href">3</a>')
    assert hrefs == ["a", "b#f"]


def test_head_elements_and_implicit_body():
    html, _ = normalize("<title>T</title><meta charset=utf-8><p>text</p>")
    assert html == ('<html>\n <head>\n  <title>T</title>\n  <meta charset="utf-8">\n </head>\n <body>\n'
                    '  <p>text</p>\n </body>\n</html>')


def test_escaping_and_boolean_attributes():
    html, _ = normalize('<p title="a &quot;q&quot; &amp; b">1 &lt; 2 &amp; 3 &gt; 0</p><input disabled checked="">')
    assert '<p title="a &quot;q&quot; &amp; b">1 &lt; 2 &amp; 3 &gt; 0</p>' in html
    assert "<input disabled checked>" in html


def test_implied_end_tags_and_unmatched_end_tags():
    doc, _ = parse("<ul><li>a<li>b</ul><p>x<div>y</div></span>")
    body = doc.children[0].children[1]
    assert [c.tag for c in body.children] == ["ul", "p", "div"]
    assert [c.tag for c in body.children[0].children] == ["li", "li"]


def test_whitespace_collapsed_except_in_pre_and_scripts_verbatim():
    html, _ = normalize("<p>a   b\n\n c</p><pre>  x\n   y</pre><script>if (a < b) { x(); }</script>")
    assert "<p>a b c</p>" in html
    assert "<pre>  x\n   y</pre>" in html
    assert "<script>if (a < b) { x(); }</script>" in html


def test_doctype_and_comments():
    html, _ = normalize("<!DOCTYPE html><html><body><!-- note --><p>x</p></body></html>")
    assert html.startswith("<!doctype html>\n<html>")
    assert "<!-- note -->" in html
