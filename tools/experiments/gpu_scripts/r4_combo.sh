#!/bin/bash
# r4_tests.sh, then (only if it ended normally: all passed, or a test failed) r4_decode.sh
bash tools/gpu/r4_tests.sh; rc=$?; echo "TESTS_RC=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu/r4_decode.sh
