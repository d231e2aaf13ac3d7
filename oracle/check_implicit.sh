#!/bin/sh
# TEST INFRASTRUCTURE: fails the _ref build when a reference TU calls a function it never declared,
# unless that name is on the TU's allowlist (oracle/Makefile passes it; DESIGN.md §4 lists each entry
# with the reference line that declares it).  usage: check_implicit.sh <file.diag> [allowed names...]
diag=$1; shift
bad=0
for n in $(grep -o "implicit declaration of function '[^']*'" "$diag" | sed "s/.*'\(.*\)'/\1/" | sort -u); do
  ok=0
  for a in "$@"; do [ "$n" = "$a" ] && ok=1; done
  if [ $ok = 0 ]; then echo "$diag: '$n' is called undeclared and is not on the allowlist" >&2; bad=1; fi
done
exit $bad
