"""Version constant (reference: modules/version/version.go:3-5)."""
VERSION = "0.1.0"
APP_NAME = "k8s-gpu-device-plugin"
