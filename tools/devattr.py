"""Diagnostic: HIP device attributes that bound occupancy (LDS, registers, waves)."""
import ctypes
h = ctypes.CDLL("libamdhip64.so")
names = {"MaxSharedMemoryPerMultiprocessor": 74, "SharedMemPerBlockOptin": None}
v = ctypes.c_int()
for nm in ("hipDeviceAttributeMaxSharedMemoryPerMultiprocessor", "hipDeviceAttributeMaxSharedMemoryPerBlock",
           "hipDeviceAttributeMaxRegistersPerMultiprocessor", "hipDeviceAttributeMaxThreadsPerMultiProcessor",
           "hipDeviceAttributeMultiprocessorCount"):
    pass
import torch
p = torch.cuda.get_device_properties(0)
print({k: getattr(p, k) for k in dir(p) if not k.startswith("_") and isinstance(getattr(p, k), (int, str))})
