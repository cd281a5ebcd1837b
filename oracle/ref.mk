# oracle/_ref: the reference's header-only QMC / fast-math layer compiled
# from /root/reference/include where it lies, with the survey build's flags
# (CMakeLists.txt:239 release flags, :336-342 FAST_MATH / FAST_TRIG), and
# linked into our own checker (ref_check.cc). No reference build system, no
# generated header, no stand-ins: only utilities/mcqmc.h,
# utilities/mathOptimizations.h, utilities/math_utils.h and yafray_constants.h
# are needed. Outputs go to oracle/_ref/ only (gitignored). Built only where
# /root/reference exists; the GPU box uses the committed fixtures instead.
REF ?= /root/reference
CXX ?= g++
OUTDIR = _ref
REFFLAGS = -O3 -ffast-math -DFAST_MATH -DFAST_TRIG -std=c++17 -I$(REF)/include

all: $(OUTDIR)/ref_check

$(OUTDIR)/ref_check: ref_check.cc
	@mkdir -p $(OUTDIR)
	$(CXX) $(REFFLAGS) -o $@ $< -ldl

clean:
	rm -rf $(OUTDIR)

.PHONY: all clean
