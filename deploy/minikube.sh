#!/usr/bin/env bash
# Local cluster for the Foremast bundle (reference: deploy/minikube.sh).
# The custom-metrics adapter (40-custom-metrics.yaml) needs webhook token
# authentication on the kubelet; the brain itself needs MI355X nodes
# (amd.com/gpu), so on a laptop run it with --nproc-per-node=1 on the CPU
# (gloo) or point FOREMAST_STORE at a brain running elsewhere.
set -euo pipefail
minikube start \
  --kubernetes-version="${K8S_VERSION:-v1.30.0}" \
  --cpus="${CPUS:-4}" \
  --memory="${MEMORY:-8192}" \
  --extra-config=kubelet.authentication-token-webhook=true \
  --extra-config=kubelet.authorization-mode=Webhook
# The recording rules (22-recording-rules.yaml, a PrometheusRule) and the
# scrape annotations need the Prometheus operator (the reference vendors the
# coreos bundle under deploy/prometheus-operator/).  Point KUBE_PROMETHEUS at
# a kube-prometheus checkout to install it first.
if [ -n "${KUBE_PROMETHEUS:-}" ]; then
  kubectl apply --server-side -f "$KUBE_PROMETHEUS/manifests/setup"
  kubectl wait --for condition=Established --all CustomResourceDefinition --namespace=monitoring
  kubectl apply -f "$KUBE_PROMETHEUS/manifests/"
fi
python -m foremast_amd.cli manifests deploy/foremast
kubectl apply -f deploy/foremast/00-namespace.yaml -f deploy/foremast/10-crds.yaml
kubectl apply -f deploy/foremast/
