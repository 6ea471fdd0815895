"""Crafted scene files that exercise TraiterFichierDeScene's quirks
(Scene.cpp:231-501).  Inputs of tests/test_host_scene.py; their expected
post-Pretraitement state is tests/golden/loader_quirks.npz, made from the
reference build by tests/golden/make_loader_golden.py."""

QUIRK_RES = (40, 30)

QUIRKS = {
    # indented comment lines are NOT comments (Trim result discarded, Scene.cpp:254);
    # this one carries 'color:' inside a surface, with a failing %i -> stale R,G,B
    "stale_rgb": """background: 10 20 30
Plane: p
  v_linear: 0 1 0
  v_const: 45
  color: 100 150 200
Quad: q
  v_quad: 1 1 1
  v_const: -100
     * --- color: R G B ---
Lumiere: l
  position: 10 100 10
  intens: 0.9
  color: 255 128 0
""",
    # keywords match anywhere; 'Poly:' inside a line starts a triangle
    "substring_keywords": """origin: 0 0 300
eye: 0 0 0
xx Poly: t1
  point: 0 -50 -50 0
  point: 1 50 -50 0
  point: 2 0 50 0
  color: 200 20 20
  rotate: 10 20 30
  translate: 1 2 3
  scale: 2 1 0.5
Lumiere: l
  position: 0 0 400
  intens: 1
""",
    # last line without a trailing newline; CRLF line endings
    "crlf_no_eol": "background: 1 2 3\r\nPlane: p\r\n  v_linear: 0 1 0\r\n  v_const: 45\r\n  color: 9 9 9",
    # stale Val0..2: 'ambient:' with no number reuses the previous float
    "stale_float": """Quad: s
  v_quad: 1 1 1
  v_const: -400
  diffus: 0.25
  ambient:
  specular: 0.5 12
  refract: 0.5 1.3
  reflect: 0.7
Lumiere: l
  position: 0 300 300
  intens: 1
""",
    # octal/hex through %i, exactly like the reference's sscanf
    "octal_hex": """background: 010 0x10 7
Poly: t
  point: 0 0 0 0
  point: 1 1 0 0
  point: 2 0 1 0
  color: 0x7f 017 255
""",
    # transforms on every kind: the plane's normal takes the translation
    # (Plan.cpp:101-114), the quadric goes through M^-1 Q M^-T
    # (Quadrique.cpp:110-146), rotations through cosf/sinf (Matrice4.h:362-422)
    "transforms_all_kinds": """origin: 30 40 260
eye: 0 10 0
up: 0.1 1 0
Plane: p
  v_linear: 0 1 0.2
  v_const: 40
  rotate: 5 -10 15
  translate: 3 -7 11
  scale: 1.5 0.75 2
  color: 90 180 45
Quad: q
  v_quad: 1 0.5 2
  v_mixte: 0.1 0 0.3
  v_linear: 2 0 -1
  v_const: -900
  rotate: 30 45 60
  translate: -5 12 4
  scale: 0.5 2 1.25
  color: 255 10 100
  specular: 0.4 20
Poly: t
  point: 0 -40 0 -30
  point: 1 40 0 -30
  point: 2 0 50 -30
  scale: 1 1 1
  rotate: 0 90 0
  color: 12 34 56
Lumiere: l
  position: -60 200 120
  intens: 0.75
  color: 200 220 255
""",
    # tabs and several spaces between values; tabs before keywords
    "tabs_and_spaces": "origin:\t0  50\t\t300\neye: 0 0 0\n\tPoly:\tt\n\tpoint:\t0\t-20 -20 0\n"
                       "  point:   1   20  -20   0\n\tpoint: 2\t0 20 0\n\tcolor:\t255\t0  9\n"
                       "Lumiere: l\n\tposition: 0 0 100\n\tintens:\t0.5\n",
    # a line whose FIRST character is '*' is a comment (Scene.cpp:258), even
    # with a surface keyword in it: no surface is made, and the point /
    # colour lines that follow apply to nothing; property lines before any
    # object are scene lines
    "comment_keywords": """* origin: 1 2 3
diffus: 0.4
*  Poly: not-a-comment
  point: 0 1 1 1
  point: 1 2 1 1
  point: 2 1 2 1
*  color: 5 6 7
Lumiere: l
  position: 5 5 5
""",
}
