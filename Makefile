# Build of the MI355X backend (HIP, gfx950) and of the CPU oracle.
#   make            -> product library + oracle
#   make ref        -> oracle/_ref (reference rigid sources; needs /root/reference)
PKG      := little-physics-engine_amd
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
# Parity flags: no FMA contraction, correctly rounded fp32 div/sqrt, IEEE denormals.
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off \
            -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero \
            -Wall -Wno-unused-function
CC       ?= gcc
CXX      ?= g++
OFLAGS   := -O2 -fPIC -ffp-contract=off -Wall -fopenmp

HIP_SRC  := $(wildcard $(PKG)/csrc/*.hip)
HIP_HDR  := $(wildcard $(PKG)/csrc/*.h) include/lpe.h
HIP_OBJ  := $(patsubst $(PKG)/csrc/%.hip,build/%.o,$(HIP_SRC))
LIB      := $(PKG)/liblpe_hip.so

ORC_SRC  := $(wildcard oracle/*.c)
ORX_SRC  := $(filter-out oracle/ref_driver.cpp,$(wildcard oracle/*.cpp))
ORACLE   := oracle/liblpe_oracle.so

all: $(LIB) $(ORACLE)

build/%.o: $(PKG)/csrc/%.hip $(HIP_HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(HIP_OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

build/oracle/%.o: oracle/%.c oracle/*.h include/lpe.h
	@mkdir -p build/oracle
	$(CC) -std=c11 $(OFLAGS) -c $< -o $@

build/oracle/%.opp: oracle/%.cpp oracle/*.h include/lpe.h
	@mkdir -p build/oracle
	$(CXX) -std=c++17 $(OFLAGS) -c $< -o $@

$(ORACLE): $(patsubst oracle/%.c,build/oracle/%.o,$(ORC_SRC)) $(patsubst oracle/%.cpp,build/oracle/%.opp,$(ORX_SRC))
	$(CXX) -shared -fPIC -fopenmp -o $@ $^ -lm

# C++ host mirror of the reference's system plugins (Systems::FluidSystem,
# RigidBodyCollisionSystem, the integrator systems) over the C ABI.  It is the
# drop-in for src/systems/, so it compiles against the reference's own headers
# (components, ISystem, EnTT): built only where /root/reference exists; the
# .so travels to the GPU box with the tree.
REF      ?= /root/reference
HOSTDIR  := $(PKG)/host
HOST_SRC := $(HOSTDIR)/lpe_backend.cpp $(wildcard $(HOSTDIR)/src/systems/*.cpp) \
            $(wildcard $(HOSTDIR)/src/systems/*/*.cpp)
HOST_HDR := $(HOSTDIR)/lpe_backend.hpp $(wildcard $(HOSTDIR)/include/systems/*/*.hpp) include/lpe.h
HOST_OBJ := $(patsubst $(HOSTDIR)/%.cpp,build/host/%.o,$(HOST_SRC))
HOSTLIB  := $(HOSTDIR)/liblpe_systems.so
HOSTFLAGS := -std=c++17 -O2 -fPIC -ffp-contract=off -Wall -Wno-unused-variable -include algorithm \
            -I$(HOSTDIR)/include -I$(HOSTDIR) -Iinclude -I$(REF)/include -I$(REF)/vendor/entt/include

build/host/%.o: $(HOSTDIR)/%.cpp $(HOST_HDR)
	@mkdir -p $(dir $@)
	$(CXX) $(HOSTFLAGS) -c $< -o $@

$(HOSTLIB): $(HOST_OBJ) $(LIB)
	$(CXX) -shared -fPIC -o $@ $(HOST_OBJ) -L$(PKG) -llpe_hip -Wl,-rpath,'$$ORIGIN/..' -Wl,-rpath,/opt/rocm/lib

host: $(HOSTLIB)

ref: host
	$(MAKE) -f oracle/Makefile.ref

# AddressSanitizer + UndefinedBehaviorSanitizer builds of the CPU side
# (SURVEY.md §5): the oracle (the checker every GPU test compares against),
# the reference's own rigid sources + driver (oracle/_ref) and the C++ host
# mirror with its EnTT harness.  Host code only (no device code is
# instrumented).  tests/test_sanitizers.py runs the CPU checks against them.
SANFLAGS := -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined
SAN      := build/asan
SAN_ORC  := $(patsubst oracle/%.c,$(SAN)/oracle/%.o,$(ORC_SRC)) $(patsubst oracle/%.cpp,$(SAN)/oracle/%.opp,$(ORX_SRC))

$(SAN)/oracle/%.o: oracle/%.c oracle/*.h include/lpe.h
	@mkdir -p $(dir $@)
	$(CC) -std=c11 $(OFLAGS) $(SANFLAGS) -c $< -o $@

$(SAN)/oracle/%.opp: oracle/%.cpp oracle/*.h include/lpe.h
	@mkdir -p $(dir $@)
	$(CXX) -std=c++17 $(OFLAGS) $(SANFLAGS) -c $< -o $@

$(SAN)/liblpe_oracle.so: $(SAN_ORC)
	$(CXX) -shared -fPIC -fopenmp $(SANFLAGS) -o $@ $^ -lm

SAN_HOST_OBJ := $(patsubst $(HOSTDIR)/%.cpp,$(SAN)/host/%.o,$(HOST_SRC))

$(SAN)/host/%.o: $(HOSTDIR)/%.cpp $(HOST_HDR)
	@mkdir -p $(dir $@)
	$(CXX) $(HOSTFLAGS) $(SANFLAGS) -c $< -o $@

$(SAN)/liblpe_systems.so: $(SAN_HOST_OBJ) $(LIB)
	$(CXX) -shared -fPIC $(SANFLAGS) -o $@ $(SAN_HOST_OBJ) -L$(PKG) -llpe_hip \
	    -Wl,-rpath,$(abspath $(PKG)) -Wl,-rpath,/opt/rocm/lib

asan: $(SAN)/liblpe_oracle.so
	@if [ -d "$(REF)/src" ]; then $(MAKE) $(SAN)/liblpe_systems.so && \
	    $(MAKE) -f oracle/Makefile.ref sanitized; fi

clean:
	rm -rf build $(LIB) $(ORACLE) $(HOSTLIB) oracle/_ref

.PHONY: all ref host clean asan
