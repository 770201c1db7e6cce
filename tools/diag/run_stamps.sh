#!/bin/bash
cd "$(dirname "$0")/../.."
FETODE_LIB=$PWD/fet-ode_amd/libfetode_stamps.so timeout -k 10 300 python tools/diag/stamps.py
