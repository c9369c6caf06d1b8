# Build recipe for the MI355X engine, the offline model converter and the CPU oracle.
#   make            -> everything below (used by __graft_entry__.build())
#   make model      -> convert the reference's archives (needs /root/reference)
HIPCC     ?= /opt/rocm/bin/hipcc
CXX       ?= g++
ARCH      ?= gfx950
PKG       := face_alignment_cvpr_2012_amd
CSRC      := $(PKG)/csrc
REFERENCE ?= /root/reference

HIPFLAGS  := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Iinclude $(EXTRA)
CXXFLAGS  := -O2 -std=c++17 -fPIC -ffp-contract=off -Wall -Iinclude

LIB       := $(PKG)/lib/libffd.so
CONVERT   := $(PKG)/bin/ffd_convert
SYNTH     := $(PKG)/bin/ffd_synth_forest
ORACLE    := oracle/build/libffd_oracle.so
MODEL     := model/ffd_model.bin
EXAMPLE   := examples/build/analyze_face
EXAMPLE2  := examples/build/estimate
EXAMPLE3  := examples/build/bench_host
EXAMPLE4  := examples/build/evaluate_mt
EXAMPLE5  := examples/build/reference_main

HIP_OBJS  := $(PKG)/lib/ffd_kernels.o $(PKG)/lib/ffd_engine.o $(PKG)/lib/ffd_group.o $(PKG)/lib/ffd_archive.o \
             $(PKG)/lib/ffd_haar.o $(PKG)/lib/ffd_detect.o $(PKG)/lib/ffd_train_k.o $(PKG)/lib/ffd_train.o \
             $(PKG)/lib/ffd_convert.o
HDRS      := include/ffd.h include/ffd_numerics.h include/ffd_gabor.h include/ffd_model_format.h $(CSRC)/ffd_device.hpp \
             $(CSRC)/ffd_kernels.hpp $(CSRC)/model_io.hpp $(CSRC)/ffd_engine_impl.hpp $(CSRC)/ffd_haar.hpp

all: $(LIB) $(CONVERT) $(SYNTH) $(ORACLE) $(EXAMPLE) $(EXAMPLE2) $(EXAMPLE3) $(EXAMPLE4) $(EXAMPLE5)

$(PKG)/lib/ffd_kernels.o: $(CSRC)/ffd_kernels.hip $(HDRS)
	@mkdir -p $(@D)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(PKG)/lib/ffd_engine.o: $(CSRC)/ffd_engine.cpp $(HDRS)
	@mkdir -p $(@D)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# host-only (the archive writer): plain g++
$(PKG)/lib/ffd_archive.o: $(CSRC)/ffd_archive.cpp include/ffd.h include/ffd_model_format.h $(CSRC)/model_io.hpp
	@mkdir -p $(@D)
	$(CXX) $(CXXFLAGS) -Iinclude -c $< -o $@

# the archive converter (ffd_model_convert) in the library; the CLI below is the same file with main()
$(PKG)/lib/ffd_convert.o: $(CSRC)/ffd_convert.cpp $(CSRC)/model_io.hpp include/ffd_model_format.h include/ffd.h
	@mkdir -p $(@D)
	$(CXX) $(CXXFLAGS) -Iinclude -c $< -o $@

$(PKG)/lib/ffd_haar.o: $(CSRC)/ffd_haar.hip $(CSRC)/ffd_haar.hpp
	@mkdir -p $(@D)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(PKG)/lib/ffd_detect.o: $(CSRC)/ffd_detect.cpp $(HDRS)
	@mkdir -p $(@D)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(PKG)/lib/ffd_train_k.o: $(CSRC)/ffd_train.hip $(CSRC)/ffd_train.hpp include/ffd_numerics.h include/ffd_gabor.h
	@mkdir -p $(@D)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(PKG)/lib/ffd_train.o: $(CSRC)/ffd_train.cpp $(CSRC)/ffd_train.hpp $(HDRS)
	@mkdir -p $(@D)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(PKG)/lib/ffd_group.o: $(CSRC)/ffd_group.cpp $(HDRS)
	@mkdir -p $(@D)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# RCCL (multi-device gather, ffd_group.cpp): the system librccl.so.1; in a process where PyTorch
# already loaded its bundled librccl.so.1 (same soname) the loader reuses that one
$(LIB): $(HIP_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(HIP_OBJS) -L/opt/rocm/lib -lrccl

$(SYNTH): $(CSRC)/ffd_synth_forest.cpp $(CSRC)/model_io.hpp include/ffd_model_format.h
	@mkdir -p $(@D)
	$(CXX) $(CXXFLAGS) -o $@ $<

$(CONVERT): $(CSRC)/ffd_convert.cpp $(CSRC)/model_io.hpp include/ffd_model_format.h include/ffd.h
	@mkdir -p $(@D)
	$(CXX) $(CXXFLAGS) -DFFD_CONVERT_MAIN -o $@ $<

$(ORACLE): oracle/ffd_oracle.cpp oracle/ffd_train_oracle.cpp oracle/ffd_oracle.h include/ffd_numerics.h include/ffd_gabor.h include/ffd_model_format.h
	@mkdir -p $(@D)
	$(CXX) $(CXXFLAGS) -shared -pthread -o $@ oracle/ffd_oracle.cpp oracle/ffd_train_oracle.cpp

model: $(CONVERT)
	@mkdir -p model
	$(CONVERT) $(REFERENCE) $(MODEL)

clean:
	rm -rf $(PKG)/lib $(PKG)/bin oracle/build

.PHONY: all model clean

$(EXAMPLE): examples/analyze_face.cpp include/FaceForest.hpp include/ffd.h $(LIB)
	@mkdir -p $(@D)
	$(CXX) -O2 -std=c++17 -Wall -Iinclude -o $@ $< -L$(PKG)/lib -lffd -Wl,-rpath,'$$ORIGIN/../../$(PKG)/lib'
$(EXAMPLE2): examples/estimate.cpp include/FaceForest.hpp include/ffd.h $(LIB)
	@mkdir -p $(@D)
	$(CXX) -O2 -std=c++17 -Wall -Iinclude -o $@ $< -L$(PKG)/lib -lffd -Wl,-rpath,'$$ORIGIN/../../$(PKG)/lib'
$(EXAMPLE3): examples/bench_host.cpp include/FaceForest.hpp include/ffd.h $(LIB)
	@mkdir -p $(@D)
	$(CXX) -O2 -std=c++17 -Wall -Iinclude -o $@ $< -L$(PKG)/lib -lffd -Wl,-rpath,'$$ORIGIN/../../$(PKG)/lib'
$(EXAMPLE4): examples/evaluate_mt.cpp include/FaceForest.hpp include/ffd.h $(LIB)
	@mkdir -p $(@D)
	$(CXX) -O2 -std=c++17 -Wall -pthread -Iinclude -o $@ $< -L$(PKG)/lib -lffd -Wl,-rpath,'$$ORIGIN/../../$(PKG)/lib'
$(EXAMPLE5): examples/reference_main.cpp include/FaceForest.hpp include/ffd.h $(LIB)
	@mkdir -p $(@D)
	$(CXX) -O2 -std=c++17 -Wall -Iinclude -o $@ $< -L$(PKG)/lib -lffd -Wl,-rpath,'$$ORIGIN/../../$(PKG)/lib'
example: $(EXAMPLE) $(EXAMPLE2) $(EXAMPLE3) $(EXAMPLE4) $(EXAMPLE5) $(EXAMPLE5)
.PHONY: example
