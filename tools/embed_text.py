"""Writes a C++ raw-string definition of a text file (the JIT kernels' device prelude): embed_text.py NAME FILE."""
import sys

name, path = sys.argv[1], sys.argv[2]
text = open(path).read()
assert ")HYJIT" not in text
sys.stdout.write(f'static const char {name}[] = R"HYJIT({text})HYJIT";\n')
