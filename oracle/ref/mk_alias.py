"""TEST INFRASTRUCTURE ONLY (oracle/_ref build recipe, development container).

The reference was written for MSVC on Windows: its #include names use backslashes and do not
always match the files' case ("Core\\PBR.h", "core\\Spectrum.h", "Core\\interaction.h").  This
script scans the reference's sources where they lie and creates, under OUT, a symlink named by
each include string that does not resolve as written, pointing at the real header it means.  With
-I OUT the sources compile unmodified; nothing is copied and no header is written.

    python oracle/ref/mk_alias.py /root/reference oracle/_ref/inc
"""
import os
import re
import sys

REF, OUT = sys.argv[1], sys.argv[2]
os.makedirs(OUT, exist_ok=True)
files = {}
for d, _, fs in os.walk(REF):
    for f in fs:
        p = os.path.join(d, f)
        files[os.path.relpath(p, REF).lower()] = p
made = 0
for d, _, fs in os.walk(REF):
    for f in fs:
        if not f.endswith((".h", ".cpp")):
            continue
        for m in re.finditer(r'#\s*include\s*[<"]([^>"]+)[>"]', open(os.path.join(d, f), errors="replace").read()):
            name = m.group(1)
            if os.path.exists(os.path.join(REF, name)):
                continue
            target = files.get(name.replace("\\", "/").lower())
            if target is None:
                continue            # a system header
            link = os.path.join(OUT, name)   # a backslash is an ordinary file-name character here
            os.makedirs(os.path.dirname(link) or OUT, exist_ok=True)
            if not os.path.lexists(link):
                os.symlink(target, link)
                made += 1
print(f"{made} include aliases in {OUT}")
