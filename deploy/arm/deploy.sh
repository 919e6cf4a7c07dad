#!/usr/bin/env bash
# Deploy dxa to Azure: AMD Instinct GPU scale set + Event Hubs (Kafka endpoint) + Blob + Key Vault + Redis + Cosmos DB
# + Application Insights (the reference's DeploymentCloud/Deployment.DataX/deploy.bat + Resource-Template.json).
#   ./deploy.sh <resource-group> <location> [parameters file]
set -euo pipefail
RG=${1:?resource group}; LOC=${2:?location}; PARAMS=${3:-$(dirname "$0")/azuredeploy.parameters.json}
az group create --name "$RG" --location "$LOC" --output none
az deployment group validate --resource-group "$RG" --template-file "$(dirname "$0")/azuredeploy.json" \
  --parameters @"$PARAMS" --output none
az deployment group create --resource-group "$RG" --template-file "$(dirname "$0")/azuredeploy.json" \
  --parameters @"$PARAMS" --query properties.outputs
