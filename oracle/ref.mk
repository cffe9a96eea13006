# oracle/ref.mk -- builds oracle/_ref/libdbow2ref.so from the reference's own
# DUtils / DBoW2 sources, compiled UNMODIFIED where they lie under
# /root/reference (TEST INFRASTRUCTURE ONLY; outputs only into oracle/_ref/,
# which is git-ignored and travels to the GPU box like our own .so files).
# Only the files that need nothing beyond the C++ standard library are used;
# see ref_shim.cpp for the list and for what is restated instead.
#   make -f ref.mk        (from oracle/; a no-op when /root/reference is absent)
REF ?= /root/reference/ORB-SLAM2/Thirdparty/DBoW2
CXX ?= g++
CXXFLAGS ?= -O2 -std=c++11 -fPIC -w
SRCS := $(REF)/DUtils/Random.cpp $(REF)/DUtils/Timestamp.cpp $(REF)/DBoW2/BowVector.cpp $(REF)/DBoW2/FeatureVector.cpp

ifneq ($(wildcard $(REF)/DUtils/Random.cpp),)
all: _ref/libdbow2ref.so
_ref/libdbow2ref.so: $(SRCS) ref_shim.cpp
	@mkdir -p _ref
	$(CXX) $(CXXFLAGS) -I$(REF) -shared -o $@ ref_shim.cpp $(SRCS)
else
all:
	@echo "reference sources not present: oracle/_ref not rebuilt"
endif
.PHONY: all
