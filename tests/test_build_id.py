"""nrx_build_id hashes the code, not the comments: a comment-only edit of a
source keeps the id, a code edit changes it (neural_rx_amd/build.py hash_sources)."""
from neural_rx_amd import build


SRC = '''// kernel comment
#include "x.h"   /* trailing */
__global__ void k(int* p) {   // body
  const char* s = "// not a comment /* nor this */";
  p[0] = 1;  /* one
               two */
  char q = '/';
}
'''


def test_comment_edit_keeps_id():
    base = build.hash_sources({"a.hip": SRC})
    edited = SRC.replace("// kernel comment", "// kernel comment, reworded\n// and a new line")
    edited = edited.replace("/* trailing */", "/* trailing, longer */").replace("two */", "two three */")
    assert build.hash_sources({"a.hip": edited}) == base


def test_code_edit_changes_id():
    base = build.hash_sources({"a.hip": SRC})
    assert build.hash_sources({"a.hip": SRC.replace("p[0] = 1;", "p[0] = 2;")}) != base
    # text inside a string literal is code
    assert build.hash_sources({"a.hip": SRC.replace("nor this", "nor that")}) != base
    assert build.hash_sources({"b.hip": SRC}) != base


def test_tree_hash_is_stable():
    assert build.source_hash() == build.source_hash()
    assert len(build.source_hash()) == 16
